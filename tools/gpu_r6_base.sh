set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 240 python tools/act_phases.py --envs 8192 --steps 30 > gpurun_out/r6a_phases.log 2>&1 || exit 3
tail -5 gpurun_out/r6a_phases.log
timeout -k 10 240 python tools/learner_only.py --active 0.023 --steps 10 > gpurun_out/r6a_lo.log 2>&1 || exit 4
tail -3 gpurun_out/r6a_lo.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r6a_bench.log 2>&1 || exit 5
tail -1 gpurun_out/r6a_bench.log | cut -c1-900
