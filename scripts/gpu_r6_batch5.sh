#!/bin/bash
# Round 6, batch 5: the NN round kernel v2 (tests vs the fp32 reference at forms 1 and 2,
# per-round time of v1 / v2 at S = 16 and S = 512, the P = 16 learner rate) and the phase
# cycles of the MultiClassPA scan.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
O=$R/gpurun_out/r6/b5
mkdir -p $O
for f in 1 2; do
  OMLDM_MLP_FORM=$f timeout -k 10 300 python -u -m pytest tests/test_kernels_dense.py -m gpu -k mlp -x -q \
    --timeout 120 --timeout-method thread > $O/mlp_tests_f$f.txt 2>&1 || { tail -30 $O/mlp_tests_f$f.txt; exit 3; }
  tail -1 $O/mlp_tests_f$f.txt
done
for f in 0 1 2; do
  timeout -k 10 60 ./.probe/mlpp 16 0 $f > $O/mlpp_s16_f$f.txt 2>&1 || { cat $O/mlpp_s16_f$f.txt; exit 3; }
  timeout -k 10 60 ./.probe/mlpp 512 0 $f > $O/mlpp_s512_f$f.txt 2>&1 || { cat $O/mlpp_s512_f$f.txt; exit 3; }
  head -1 $O/mlpp_s16_f$f.txt; head -1 $O/mlpp_s512_f$f.txt
done
cat $O/mlpp_s16_f0.txt
for f in 0 1 2; do
  OMLDM_MLP_FORM=$f timeout -k 10 240 python bench/learners.py --preset p16 --steps 10 --only NN > $O/nn_p16_f$f.json 2>&1 || { tail -20 $O/nn_p16_f$f.json; exit 3; }
  tail -c 400 $O/nn_p16_f$f.json
done
timeout -k 10 600 python -u -m pytest tests/test_scan3.py -m gpu -k multiclass -x -v --timeout 300 --timeout-method thread > $O/mc_tests.txt 2>&1 || { tail -40 $O/mc_tests.txt; exit 3; }
tail -3 $O/mc_tests.txt
for k in 4 10 16; do
  timeout -k 10 240 python scripts/mc_diag.py --classes $k > $O/mc_diag_k$k.json 2>&1 || { tail -20 $O/mc_diag_k$k.json; exit 3; }
  cat $O/mc_diag_k$k.json
done
mkdir -p gpurun_out/r6/async
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u bench/async_rehearsal.py --seconds 3 > gpurun_out/r6/async/rehearsal_fa.json 2> gpurun_out/r6/async/rehearsal_fa.err || { tail -20 gpurun_out/r6/async/rehearsal_fa.err; exit 3; }
timeout -k 10 400 python -u bench/async_rehearsal.py --seconds 3 --slow 2 > gpurun_out/r6/async/rehearsal_fa_slow.json 2> gpurun_out/r6/async/rehearsal_fa_slow.err || { tail -20 gpurun_out/r6/async/rehearsal_fa_slow.err; exit 3; }
cut -c 1-3000 gpurun_out/r6/async/rehearsal_fa.json
