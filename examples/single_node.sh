#!/bin/bash
# One node, file-backed topics, every GPU a rank (the reference's recipe, README.md:20-41:
# create the topics, start the job, send requests and data, read the answers).
set -eu
T=${TOPICS:-/tmp/omldm_topics}
NGPU=${NGPU:-1}
N=${N:-200000}
rm -rf "$T" && mkdir -p "$T"
python -m omldm_amd.tools topics --bootstrap "file://$T" --data-partitions 8
python -m omldm_amd.tools synth --bootstrap "file://$T" --topic trainingData --n "$N"
cat > "$T/requests.jsonl" <<'REQ'
{"id": 1, "request": "Create", "learner": {"name": "SVM", "hyperParameters": {"C": 1.0}}, "preProcessors": [{"name": "StandardScaler"}], "trainingConfiguration": {"protocol": "Synchronous"}}
{"id": 2, "request": "Create", "learner": {"name": "ORR", "hyperParameters": {"lambda": 1.0}}, "preProcessors": [{"name": "PolynomialFeatures", "hyperParameters": {"degree": 2}}], "trainingConfiguration": {"protocol": "FGM"}}
{"id": 1, "request": "Query", "requestId": 7}
REQ
python -m omldm_amd.tools produce --bootstrap "file://$T" --topic requests --file "$T/requests.jsonl"
ADDR=()
for k in trainingDataAddr forecastingDataAddr requestsAddr responsesAddr predictionsAddr performanceAddr; do
  ADDR+=(--$k "file://$T")
done
# the job ends itself after --timeout ms without new records (the reference's idle rule)
torchrun --nnodes 1 --nproc-per-node "$NGPU" --master-addr 127.0.0.1 --master-port ${PORT:-29511} \
  -m omldm_amd "${ADDR[@]}" --parallelism "$NGPU" --timeout 3000
python -m omldm_amd.tools tail --bootstrap "file://$T" --topic responses -n 3
python -m omldm_amd.tools tail --bootstrap "file://$T" --topic performance -n 1
