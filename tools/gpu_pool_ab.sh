# Pool-backward kernel check + A/B (2x2-block vs output-order form), then the full GPU check.
#   bash tools/gpu_pool_ab.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-pool}
timeout -k 10 240 python -u -m pytest tests/test_gpu_conv.py -k pool -q --timeout 120 \
  --timeout-method thread > gpurun_out/${tag}_pooltests.log 2>&1 || { tail -20 gpurun_out/${tag}_pooltests.log; exit 1; }
tail -1 gpurun_out/${tag}_pooltests.log
bash tools/lt_ab.sh ${tag} "MBK_POOL_BWD_OUT=0" "MBK_POOL_BWD_OUT=1" || exit 1
MBK_POOL_BWD_OUT=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench_out.log 2>&1 || exit $?
tail -1 gpurun_out/${tag}_bench_out.log | cut -c1-300
[ "${2:-full}" = quick ] && exit 0
bash tools/gpu_all.sh ${tag}
