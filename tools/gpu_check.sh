#!/bin/bash
# One gpurun session: smoke -> GPU parity tests -> bench -> rocprofv3 stats.
# Each GPU step has its own time limit; a fault, abort or timeout ends the
# session (exit codes other than 0/1 stop the chain).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="${STEPS:-smoke pytest bench prof}"
run() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
for s in $STEPS; do
  case $s in
    micro) run micro 300 tools/micro/${MICRO:-bs16_rate} ;;
    smoke) run smoke 400 python -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest) run pytest 1500 python -u -m pytest tests/ -v -m gpu -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} ;;
    bench) run bench 600 python bench.py ${BENCH_ARGS:-} ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} ;;
    pmc)
      PB="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --records ${PMC_RECORDS:-262144} ${BENCH_ARGS:-}"
      run pmc_a 600 rocprofv3 --kernel-include-regex "${PMC_KERNEL:-gcm_kernel}" --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_a -o run --output-format csv -- $PB
      run pmc_b 600 rocprofv3 --kernel-include-regex "${PMC_KERNEL:-gcm_kernel}" --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY -d gpurun_out/pmc_b -o run --output-format csv -- $PB
      run pmc_c 600 rocprofv3 --kernel-include-regex "${PMC_KERNEL:-gcm_kernel}" --pmc FETCH_SIZE -d gpurun_out/pmc_c -o run --output-format csv -- $PB
      run pmc_d 600 rocprofv3 --kernel-include-regex "${PMC_KERNEL:-gcm_kernel}" --pmc WRITE_SIZE -d gpurun_out/pmc_d -o run --output-format csv -- $PB
      ;;
    pmcx)
      # Custom counter passes: PMC_SETS="A B C;D E" (one rocprofv3 pass per set).
      PB="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --records ${PMC_RECORDS:-262144} ${BENCH_ARGS:-}"
      i=0
      IFS=';' read -ra SETS <<< "${PMC_SETS:-SQ_WAVES}"
      for set in "${SETS[@]}"; do
        i=$((i+1))
        run pmcx_$i 600 rocprofv3 --kernel-include-regex "${PMC_KERNEL:-gcm_kernel}" --pmc $set -d gpurun_out/pmcx_$i -o run --output-format csv -- $PB
      done
      ;;
    *) echo "unknown step $s" ;;
  esac
done
