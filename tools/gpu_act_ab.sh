# Fused acting step: GPU tests, then variants on the headline bench (A/B), then a timeline.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_act.py > gpurun_out/act_tests.log 2>&1 || { tail -40 gpurun_out/act_tests.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/act_tests.log | tail -6
for v in ${AB_VARIANTS:-"MBK_ACT_SPARSE=1" "MBK_ACT_SPARSE=0" "MBK_FUSED_ACT=0"}; do
  env $v timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ab.log 2>&1 || { tail -30 gpurun_out/ab.log; exit 1; }
  echo "$v $(python -c "import json,sys; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); a=d['actor_stats']; l=d['learner_phase_ms_rank0']; print(round(d['value']/1e6,3), 'gpu', a['gpu_phase_ms'], 'env', a['env_phase_ms'], 'fwd', l['fwd'], 'bwd', l['bwd'])")"
done
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/tl -o run --output-format csv \
  -- python $R/bench.py --steps 12 --warmup 4 > $R/gpurun_out/tl_bench.log 2>&1 || exit $?
python $R/tools/timeline.py /tmp/tl 0.5 > $R/gpurun_out/tl_fused.txt && cat $R/gpurun_out/tl_fused.txt
