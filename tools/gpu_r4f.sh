# One GPU call: WIDE stage-0 conv test, config 4 bench, head launch-B grid A/B on the bench.
#   bash tools/gpu_r4f.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-r4f}
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q -k conv0_row --timeout 120 --timeout-method thread \
  > gpurun_out/${tag}_conv_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_conv_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_conv_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --size 24 --arch impala_deep > gpurun_out/${tag}_c4.log 2>&1 || exit 2
python - gpurun_out/${tag}_c4.log <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("c4", r["value"], r["ms_per_step"], r.get("learner_phase_ms_rank0"))
PY
for g in 16 4 1; do
  MBK_HEAD_ACT_GRID=$g timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench_g$g.log 2>&1 || exit 3
  python - $g gpurun_out/${tag}_bench_g$g.log <<'PY'
import json, sys
r = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
a = r.get("actor_stats_per_rank", [{}])[0]
print("head_act grid per 8 CUs", sys.argv[1], r["value"], r["ms_per_step"], r.get("learner_phase_ms_rank0"), a.get("gpu_phase_ms"))
PY
done
# learner launches over 65K-image ranges (+ the policy gate): the policy step's CU access
for v in "MBK_LEARN_CHUNK=65536" "MBK_LEARN_CHUNK=65536 MBK_POLICY_GATE=1"; do
  env $v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench_lc.log 2>&1 || exit 4
  python - "$v" gpurun_out/${tag}_bench_lc.log <<'PY'
import json, sys
r = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
a = r.get("actor_stats_per_rank", [{}])[0]
print(sys.argv[1], r["value"], r["ms_per_step"], r.get("learner_phase_ms_rank0"), a.get("gpu_phase_ms"))
PY
done
# pipeline shape on the new acting kernel: 2 policy lanes, 3 / 5 groups
for v in "--lanes 2" "--groups 5" "--groups 3"; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 $v > gpurun_out/${tag}_bench_shape.log 2>&1 || exit 5
  python - "$v" gpurun_out/${tag}_bench_shape.log <<'PY'
import json, sys
r = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
a = r.get("actor_stats_per_rank", [{}])[0]
print(sys.argv[1], r["value"], r["ms_per_step"], a.get("gpu_phase_ms"), a.get("env_phase_ms"))
PY
done
