set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_agent_api.py tests/test_gpu_engine.py -q --timeout 200 --timeout-method thread > gpurun_out/t3.log 2>&1
rc=$?; tail -3 gpurun_out/t3.log; grep -E "^E |FAILED" gpurun_out/t3.log | head -20; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/microbench.py --E 8192 --learn_B "" --iters 50 > gpurun_out/t3_micro.log 2>&1 || exit $?
grep '"what"' gpurun_out/t3_micro.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/t3_bench.log 2>&1 || exit $?
tail -1 gpurun_out/t3_bench.log | cut -c1-200
