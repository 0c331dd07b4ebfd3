# Max-pool backward folded into the stage convs' wgrad / dgrad staging:
# stage 0 only (MBK_FUSED_POOL_BWD=s0), every stage (1) vs separate (0).
#   bash tools/gpu_r4n.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-r4n}
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
bash tools/lt_ab.sh ${tag} "MBK_FUSED_POOL_BWD=0" "MBK_FUSED_POOL_BWD=s0" "MBK_FUSED_POOL_BWD=1" || exit 4
grep -E "pool_bwd|wgrad_kernel<32, 16|unpool|update span" gpurun_out/${tag}_lt1.md gpurun_out/${tag}_lt2.md gpurun_out/${tag}_lt3.md
