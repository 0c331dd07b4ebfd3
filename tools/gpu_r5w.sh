# Stage-0 pool-fused weight gradient after spreading its scatter over all waves: tests + A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 200 --timeout-method thread \
  -k "pool_conv_bwd or pool_fused" > gpurun_out/r5w_tests.log 2>&1 || { tail -40 gpurun_out/r5w_tests.log; exit 1; }
tail -2 gpurun_out/r5w_tests.log
LT_ARGS="--active 0.025" bash tools/lt_ab.sh r5w "--set enc.fused_pool_wgrad0=0" "--set enc.fused_pool_wgrad0=1" \
  "--set enc.fused_pool_wgrad0=0" "--set enc.fused_pool_wgrad0=1" || exit 3
grep -E "pool_conv_bwd|pool_bwd_idx_kernel<16>|conv_wgrad_kernel<32, 16" gpurun_out/r5w_lt1.md gpurun_out/r5w_lt2.md
