# Stall-study counter passes (SQ wait / active / LDS cycles) of one command, summarised per
# kernel by tools/pmc_stalls.py into gpurun_out/<name>_wait.md.
#   bash tools/pmc_wait.sh <name> <match substr,...> <python args...>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
name=$1; shift
match=$1; shift
script=$1; shift
case $script in /*) ;; *) script=$R/$script ;; esac
cd /tmp && export TMPDIR=/tmp
ARGS=("$script" "$@")
run() {
  local d=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace -d /tmp/${name}_$d -o run \
    --output-format csv -- python "${ARGS[@]}" > $R/gpurun_out/${name}_$d.log 2>&1
}
run w1 SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES || { tail -5 $R/gpurun_out/${name}_w1.log; exit 2; }
run w2 SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA || { tail -5 $R/gpurun_out/${name}_w2.log; exit 3; }
python $R/tools/pmc_stalls.py $R/gpurun_out/${name}_wait.md /tmp/${name}_w1 /tmp/${name}_w2 --match=$match
rm -rf /tmp/${name}_w1 /tmp/${name}_w2
