set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in "3 8192" "4 8192" "2 12288" "3 12288" "4 6144" "6 4096"; do
  set -- $v
  timeout -k 10 200 python bench.py --steps 12 --warmup 4 --groups $1 --envs_per_group $2 > gpurun_out/sw.log 2>&1 || exit $?
  echo "groups=$1 E=$2 $(tail -1 gpurun_out/sw.log | grep -o '"value": [0-9.]*\|"gpu_phase_ms": [0-9.]*\|"env_phase_ms": [0-9.]*\|"fwd": [0-9.]*\|"bwd": [0-9.]*' | tr '\n' ' ')"
done
