# Same-box A/B of headline-bench variants, then the learner's per-dispatch timeline.
#   bash tools/ab_bench.sh <tag> "<ENV=.. args>" "<ENV=.. args>" ...
# Each variant is "VAR=value ... -- bench args" (either side may be empty). Stops at the first
# failing / timed-out run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; shift
mkdir -p $R/gpurun_out
cd $R
i=0
for v in "$@"; do
  envs=${v%%--*}; args=""
  [[ "$v" == *--* ]] && args=${v#*--}
  i=$((i+1))
  env $envs timeout -k 10 240 python bench.py --steps 20 --warmup 5 $args \
    > gpurun_out/${tag}_v$i.log 2>&1 || { echo "variant $i failed"; tail -5 gpurun_out/${tag}_v$i.log; exit 1; }
  python - "$v" gpurun_out/${tag}_v$i.log <<'EOF'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
a = d["actor_stats"]; l = d["learner_phase_ms_rank0"]
print(f"[{sys.argv[1]}] {d['value']/1e6:.3f}M fps, {d['ms_per_step']} ms/step, gpu_phase {a['gpu_phase_ms']} "
      f"env_phase {a['env_phase_ms']} busy {a['env_worker_busy_frac']} fwd {l.get('fwd')} bwd {l.get('bwd')}"
      + (f" step_split {d['policy_step_gpu_ms']}" if "policy_step_gpu_ms" in d else ""))
EOF
done
if [ -n "$LT" ]; then
  cd /tmp && export TMPDIR=/tmp && rm -rf /tmp/lt
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/lt -o run --output-format csv \
    -- python $R/tools/learner_only.py --steps 2 > $R/gpurun_out/${tag}_lt.log 2>&1 || exit $?
  python $R/tools/layer_times.py /tmp/lt --out $R/gpurun_out/${tag}_lt.md > /dev/null || exit $?
  tail -2 $R/gpurun_out/${tag}_lt.md
fi
