# Bench sweep over engine pipelining parameters (one GPU). Usage: bash tools/gpu_sweep.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for cfg in "2 4096 0" "3 4096 0" "4 2048 0" "4 4096 0" "2 4096 8" "3 4096 8" "6 2048 0"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --steps 20 --warmup 4 --groups $1 --envs_per_group $2 \
    --learner_cu_reserve $3 > gpurun_out/sweep2_$1_$2_$3.log 2>&1 || exit 2
done
