# One-pass FC weight + bias gradient (MBK_FC_WIDE=1) vs fc_wgrad chunks + colsum (0).
#   bash tools/gpu_r4p.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-r4p}
timeout -k 10 300 python -u -m pytest tests/test_gpu_fc.py tests/test_gpu_learner_parity.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
bash tools/lt_ab.sh ${tag} "MBK_FC_WIDE=1" "MBK_FC_WIDE=0" || exit 4
grep -E "fc_wgrad|colsum|update span" gpurun_out/${tag}_lt1.md gpurun_out/${tag}_lt2.md
