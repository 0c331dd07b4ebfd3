set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
# config 5: self-play league groups, bf16 fused acting trunk vs the fp8 per-layer trunk
for v in "" "--fp8_policy"; do
  timeout -k 10 300 python bench.py --steps 15 --warmup 4 --selfplay_groups 1 $v > gpurun_out/c5_${v:-bf16}.log 2>&1 || exit $?
  echo "c5 ${v:-bf16}: $(tail -1 gpurun_out/c5_${v:-bf16}.log | cut -c1-200)"
done
# config 4: 24x24 IMPALA-ResNet deep encoder (16/32/32/32)
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --size 24 --arch impala_deep > gpurun_out/c4.log 2>&1 || exit $?
echo "c4: $(tail -1 gpurun_out/c4.log | cut -c1-300)"
# config 2: 64 CPU actor processes -> 1 GPU learner, 10x10 GridNet
timeout -k 10 400 python tools/bench_mono.py --actors 64 --size 10 --arch gridnet --steps 10 --warmup 3 > gpurun_out/c2.log 2>&1 || exit $?
echo "c2: $(tail -1 gpurun_out/c2.log | cut -c1-300)"
bash tools/prof.sh c4_prof bench.py --steps 6 --warmup 2 --size 24 --arch impala_deep || exit $?
bash tools/prof.sh c5_prof bench.py --steps 6 --warmup 2 --selfplay_groups 1 --fp8_policy || exit $?
bash tools/prof.sh c2_prof tools/bench_mono.py --actors 64 --size 10 --arch gridnet --steps 5 --warmup 2
