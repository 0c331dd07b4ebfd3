# Round-5 kernel check: fused stage backward kernels (stage 0 pool-fused wgrad, stage 1
# pool+conv backward) and the pipelined acting trunk: their GPU tests, same-box learner A/Bs,
# the acting step's phase split.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_act.py tests/test_gpu_learner_parity.py \
  -x -q --timeout 200 --timeout-method thread -k "pool_conv_bwd or pool_fused or learner_parity or act" \
  > gpurun_out/r5v_tests.log 2>&1 || { tail -40 gpurun_out/r5v_tests.log; exit 1; }
tail -2 gpurun_out/r5v_tests.log
timeout -k 10 200 python tools/act_phases.py > gpurun_out/r5v_act.log 2>&1 || { tail -20 gpurun_out/r5v_act.log; exit 2; }
cat gpurun_out/r5v_act.log | tail -28
LT_ARGS="--active 0.025" bash tools/lt_ab.sh r5v "--set enc.fused_pool_conv_bwd=0" "--set enc.fused_pool_conv_bwd=1" \
  "--set enc.fused_pool_wgrad0=1" "--set enc.fused_pool_conv_bwd=0" "--set enc.fused_pool_conv_bwd=1" "--set enc.fused_pool_wgrad0=1" || exit 3
