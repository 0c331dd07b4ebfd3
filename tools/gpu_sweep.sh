set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 200 python tools/microbench.py --E 256,1024,4096 --learn_B 1024 > gpurun_out/micro2.log 2>&1 || exit 1
for cfg in "2 1024 1" "2 2048 1" "4 1024 1" "2 4096 1"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --steps 15 --warmup 3 --groups $1 --envs_per_group $2 --batch_slots $3 > gpurun_out/sweep_$1_$2_$3.log 2>&1 || exit 2
done
