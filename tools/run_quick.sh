set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_head.py tests/test_gpu_obs_mask.py tests/test_gpu_engine.py > gpurun_out/gt.log 2>&1 || exit $?
tail -1 gpurun_out/gt.log
for v in "X=0" "X=1"; do
  env $v timeout -k 10 200 python bench.py --steps 15 --warmup 4 > gpurun_out/sw.log 2>&1 || exit $?
  echo "$v $(tail -1 gpurun_out/sw.log | grep -o '"value": [0-9.]*\|"gpu_phase_ms": [0-9.]*\|"fwd": [0-9.]*\|"bwd": [0-9.]*' | tr '\n' ' ')"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/tl -o run --output-format csv \
  -- python $GRAFT_REPO_ROOT/bench.py --steps 12 --warmup 4 > $GRAFT_REPO_ROOT/gpurun_out/tl_bench.log 2>&1 || exit $?
python $GRAFT_REPO_ROOT/tools/timeline.py /tmp/tl 0.5 > $GRAFT_REPO_ROOT/gpurun_out/tl.txt 2>&1 || exit $?
head -20 $GRAFT_REPO_ROOT/gpurun_out/tl.txt
