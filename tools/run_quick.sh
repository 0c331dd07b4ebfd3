set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_learner_parity.py tests/test_gpu_conv.py -k "fused or parity or dx_value" > gpurun_out/t2.log 2>&1 || { tail -30 gpurun_out/t2.log; exit 1; }
tail -2 gpurun_out/t2.log
LT=1 bash tools/ab_bench.sh ab3 "" "MBK_FUSED_POOL_BWD=s0" "MBK_FUSED_POOL_BWD=1"
cd /tmp && export TMPDIR=/tmp && rm -rf /tmp/lt
MBK_FUSED_POOL_BWD=s0 timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/lt -o run --output-format csv \
    -- python $GRAFT_REPO_ROOT/tools/learner_only.py --steps 2 > $GRAFT_REPO_ROOT/gpurun_out/ab3_lts0.log 2>&1 || exit $?
python $GRAFT_REPO_ROOT/tools/layer_times.py /tmp/lt --out $GRAFT_REPO_ROOT/gpurun_out/ab3_lts0.md > /dev/null || exit $?
tail -1 $GRAFT_REPO_ROOT/gpurun_out/ab3_lts0.md
