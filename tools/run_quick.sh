set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 120 python tools/dbg/res32_check.py 4 37 2>&1 | head -4
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv.py -k "res_bwd32 or res_bwd16 or res_blk32" > gpurun_out/t3.log 2>&1 || { tail -40 gpurun_out/t3.log; exit 1; }
tail -2 gpurun_out/t3.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_learner_parity.py > gpurun_out/t3b.log 2>&1 || { tail -40 gpurun_out/t3b.log; exit 1; }
tail -2 gpurun_out/t3b.log
LT=1 bash tools/ab_bench.sh ab4 "" "MBK_FUSED_RES32=0"
