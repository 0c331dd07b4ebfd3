set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv.py -k "res_blk32 or res_fwd16" > gpurun_out/gt.log 2>&1 || { tail -30 gpurun_out/gt.log; exit 1; }
tail -1 gpurun_out/gt.log
cd /tmp && export TMPDIR=/tmp
for v in 1; do
  rm -rf /tmp/lt
  MBK_FUSED_RES_FWD32=$v timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/lt -o run --output-format csv \
    -- python $GRAFT_REPO_ROOT/tools/learner_only.py --steps 2 > $GRAFT_REPO_ROOT/gpurun_out/lt$v.log 2>&1 || exit $?
  python $GRAFT_REPO_ROOT/tools/layer_times.py /tmp/lt --out $GRAFT_REPO_ROOT/gpurun_out/lt$v.md > /dev/null || exit $?
  echo "FWD32=$v"; grep "res_\|conv_fwd\|update span" $GRAFT_REPO_ROOT/gpurun_out/lt$v.md
done
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python bench.py --steps 15 --warmup 4 > gpurun_out/sw.log 2>&1 || exit $?
tail -1 gpurun_out/sw.log
