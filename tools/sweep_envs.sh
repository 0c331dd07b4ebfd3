# Bench sweep over (env groups, envs per group) on one GPU.
#   SWEEP="2:8192 4:4096" STEPS=16 bash tools/sweep_envs.sh
set -o pipefail
mkdir -p gpurun_out
for cfg in ${SWEEP:-2:8192}; do
  g=${cfg%%:*}; e=${cfg##*:}
  timeout -k 10 300 python -u bench.py --steps ${STEPS:-16} --warmup 4 --groups $g --envs_per_group $e \
    $BENCH_ARGS > gpurun_out/sw_${g}_${e}.log 2>&1 || exit 2
  echo "$g x $e $(grep -o '"value": [0-9.]*' gpurun_out/sw_${g}_${e}.log | head -1) $(grep -o '"gpu_phase_ms": [0-9.]*' gpurun_out/sw_${g}_${e}.log) $(grep -o '"env_worker_busy_frac": [0-9.]*' gpurun_out/sw_${g}_${e}.log)"
done
