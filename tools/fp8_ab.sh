# fp8 acting trunk on the GPU box: numerics tests, isolated policy-step timing (bf16 fused /
# fp8 fused / fp8 per-layer), then the BASELINE config-5 bench A/B (self-play league group).
#   bash tools/fp8_ab.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -q -x --timeout 120 \
  --timeout-method thread -k "fp8 or fused_trunk" > gpurun_out/${tag}_pytest.log 2>&1 \
  || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -2 gpurun_out/${tag}_pytest.log
for v in "bf16:" "fp8:--fp8" "fp8_layers:--fp8"; do
  name=${v%%:*}; args=${v#*:}
  t8=1; [ "$name" = fp8_layers ] && t8=0
  MBK_TRUNK8=$t8 timeout -k 10 180 python tools/microbench.py --E 8192 --iters 50 --no_learner $args \
    > gpurun_out/${tag}_micro_$name.log 2>&1 || { tail -5 gpurun_out/${tag}_micro_$name.log; exit 1; }
  grep policy_step gpurun_out/${tag}_micro_$name.log
done
for v in "bf16:" "fp8:--fp8_policy" "fp8_layers:--fp8_policy"; do
  name=${v%%:*}; args=${v#*:}
  t8=1; [ "$name" = fp8_layers ] && t8=0
  MBK_TRUNK8=$t8 timeout -k 10 240 python bench.py --steps 20 --warmup 5 --selfplay_groups 1 $args \
    > gpurun_out/${tag}_c5_$name.log 2>&1 || { tail -5 gpurun_out/${tag}_c5_$name.log; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/${tag}_c5_$name.log $name
done
