# Round-5 learning evidence on the GPU box: the 16x16 fused-path learning test, then the
# 1.68 B-frame headline-config training run through the CLI (experiments/r5b1L), then the
# settled headline bench.
#   bash tools/gpu_learn_run.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-r5}
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_entry.py -x -v -s --timeout 280 \
  --timeout-method thread -k fused_16x16 > gpurun_out/${tag}_learn16.log 2>&1 || { tail -30 gpurun_out/${tag}_learn16.log; exit 1; }
grep -E "16x16 fused|passed|failed" gpurun_out/${tag}_learn16.log
bash tools/run_experiment.sh r5b1L 420 --runtime gpu --env_size 16 --groups 3 \
  --envs_per_group 8192 --unroll_length 64 --batch_size 1 --max_updates 3200 \
  --max_episode_steps 2000 --log_every 10 --checkpoint_every 0 || exit 2
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.log 2>&1 || exit 3
tail -1 gpurun_out/${tag}_bench.log | cut -c1-400
