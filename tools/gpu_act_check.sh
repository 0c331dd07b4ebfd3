# Fused acting step: bit-identity tests, then the headline bench with the fused step and with
# the captured-graph step (A/B), each under its own time limit.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_act.py > gpurun_out/act_tests.log 2>&1 || { tail -40 gpurun_out/act_tests.log; exit 1; }
tail -5 gpurun_out/act_tests.log
timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 > gpurun_out/act_bench_fused.log 2>&1 || { tail -30 gpurun_out/act_bench_fused.log; exit 1; }
tail -1 gpurun_out/act_bench_fused.log
MBK_FUSED_ACT=0 timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 > gpurun_out/act_bench_graph.log 2>&1 || { tail -30 gpurun_out/act_bench_graph.log; exit 1; }
tail -1 gpurun_out/act_bench_graph.log
