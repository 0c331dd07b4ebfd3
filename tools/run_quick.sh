set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_head.py tests/test_gpu_learner_parity.py tests/test_gpu_agent_api.py > gpurun_out/gt.log 2>&1 || exit $?
tail -1 gpurun_out/gt.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/lt -o run --output-format csv \
  -- python $GRAFT_REPO_ROOT/tools/learner_only.py --steps 2 > $GRAFT_REPO_ROOT/gpurun_out/lt.log 2>&1 || exit $?
python $GRAFT_REPO_ROOT/tools/layer_times.py /tmp/lt --out $GRAFT_REPO_ROOT/gpurun_out/lt.md > /dev/null || exit $?
grep "head\|row_sum\|update span" $GRAFT_REPO_ROOT/gpurun_out/lt.md
cd $GRAFT_REPO_ROOT
for v in "X=0" "X=1"; do
  env $v timeout -k 10 200 python bench.py --steps 15 --warmup 4 > gpurun_out/sw.log 2>&1 || exit $?
  echo "$v $(tail -1 gpurun_out/sw.log | grep -o '"value": [0-9.]*\|"gpu_phase_ms": [0-9.]*\|"env_phase_ms": [0-9.]*\|"fwd": [0-9.]*\|"bwd": [0-9.]*' | tr '\n' ' ')"
done
