# Acting-step check: fused-step bit identity + head tests, isolated launch timings, short bench.
#   bash tools/gpu_r6_act.sh <tag> [bench]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
tag=${1:-act}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_act.py tests/test_gpu_head.py > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 3; }
tail -3 gpurun_out/${tag}_tests.log
timeout -k 10 240 python tools/act_phases.py --envs 8192 --steps 30 > gpurun_out/${tag}_phases.log 2>&1 || { tail -20 gpurun_out/${tag}_phases.log; exit 4; }
head -4 gpurun_out/${tag}_phases.log
if [ "$2" = bench ]; then
  timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 5; }
  tail -1 gpurun_out/${tag}_bench.log | cut -c1-400
  tail -1 gpurun_out/${tag}_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['actor_stats'], d['learner_phase_ms_rank0'])"
fi
