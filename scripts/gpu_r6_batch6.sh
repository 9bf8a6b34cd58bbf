#!/bin/bash
# Round 6, batch 6: NN v2 phase stamps; MultiClassPA template diagnostics (K = 8 problem on
# the 8 and 16 templates, the phase cycles at K = 4 / 8 / 16) and the scan tests.
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
O=$R/gpurun_out/r6/b6
mkdir -p $O
for f in 0 1 2; do
  timeout -k 10 60 ./.probe/mlpp 16 0 $f > $O/mlpp_s16_f$f.txt 2>&1 || { cat $O/mlpp_s16_f$f.txt; exit 3; }
  cat $O/mlpp_s16_f$f.txt
done
for args in "8 16" "4 16" "4 8" "10 16 5 300"; do
  timeout -k 10 300 python scripts/mc_kt_diag.py $args >> $O/mc_kt.txt 2>&1 || { tail -20 $O/mc_kt.txt; exit 3; }
done
cat $O/mc_kt.txt
for k in 4 8 16; do
  timeout -k 10 240 python scripts/mc_diag.py --classes $k > $O/mc_diag_k$k.json 2>&1 || { tail -20 $O/mc_diag_k$k.json; exit 3; }
  cat $O/mc_diag_k$k.json
done
