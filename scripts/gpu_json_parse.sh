set -u
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_json_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/jp_tests.log 2>&1; rc=$?; tail -3 gpurun_out/jp_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/json_parse_probe.py
