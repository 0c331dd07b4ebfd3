# configs 4 / 2 with and without the backward occupancy cap (bench.py --learner_bwd_occupancy)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-cfo}
run() {
  name=$1; shift
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 "$@" > gpurun_out/${tag}_$name.log 2>&1 || { tail -20 gpurun_out/${tag}_$name.log; exit 5; }
  grep metric gpurun_out/${tag}_$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', round(d['value']/1e6,3), 'M; lrn', d['learner_phase_ms_rank0']['fwd'], d['learner_phase_ms_rank0']['bwd'], 'ms/step', d['ms_per_step'])"
}
for occ in 0 1; do
  run c4_occ$occ --size 24 --arch impala_deep --learner_bwd_occupancy $occ
  run c2_occ$occ --size 10 --arch gridnet --learner_bwd_occupancy $occ
done
