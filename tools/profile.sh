#!/bin/bash
# Profiling evidence on one GPU: for each config in $CONFIGS the rocprofv3
# kernel stats of the bench command ("stats") and the PMC passes of its bulk
# kernel ("pmc": FETCH_SIZE, WRITE_SIZE and the SQ/GRBM busy counters, each a
# run of its own), and the end-to-end host-buffer rate ("e2e",
# tools/e2e_bench.py).  Output under $O (default gpurun_out/prof).  Each GPU
# step has its own time limit; the chain stops at the first failure.
# Summarise the PMC passes with: tools/pmc_traffic.py $O [profiles/traffic.json]
#   O=gpurun_out/r03a CONFIGS="config2 config3" PASSES="stats pmc" tools/profile.sh
# ENGINE=bs: the AES-GCM configs on the table-free engine (BSSL_AMD_GCM_MODE=bs,
# kernels gcm_bs_kernel / gcm_bs_keyset_kernel), output dirs prefixed bs_.
set -u
ENGINE=${ENGINE:-table}
EP=""
if [ "$ENGINE" = bs ]; then export BSSL_AMD_GCM_MODE=bs; EP=bs_; fi
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=${O:-gpurun_out/prof}
CONFIGS=${CONFIGS:-config2 config3 config3x config4 config5 configS}
PASSES=${PASSES:-stats pmc}
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a $O/steps.log
  [ $rc -eq 0 ] || exit $rc
}
has() { case " $PASSES " in *" $1 "*) return 0 ;; esac; return 1; }
# FETCH_SIZE / WRITE_SIZE calibration on known byte counts, one copy kernel
# per record access pattern (tools/micro/calib_copy, built in-tree here).
# Geometries: 1350-byte records at the bench's 1408-byte stride (configs G, 3,
# the short records of 4) and 16 KiB records (configs 2, 5, the long ones of 4).
if has calib; then
  for geo in "1350 1408 1048576" "16384 16384 262144"; do
    tag=$(echo $geo | tr ' ' 'x')
    step calib_run_$tag 60 tools/micro/calib_copy 3 $geo
    step calib_fetch_$tag 60 rocprofv3 --pmc FETCH_SIZE -d $O/calib_fetch_$tag -o run --output-format csv -- tools/micro/calib_copy 2 $geo
    step calib_write_$tag 60 rocprofv3 --pmc WRITE_SIZE -d $O/calib_write_$tag -o run --output-format csv -- tools/micro/calib_copy 2 $geo
  done
fi
for cfg in $CONFIGS; do
  case $cfg in config3|config3x) K=chacha_poly_kernel ;; configS) K=gcm_siv_kernel ;; config5) K=gcm_keyset_kernel ;; *) K=gcm_kernel ;; esac
  if [ "$ENGINE" = bs ]; then case $cfg in config5) K=gcm_bs_keyset_kernel ;; *) K=gcm_bs_kernel ;; esac; fi
  if has stats; then
    step ${EP}stats_$cfg 300 rocprofv3 --kernel-trace --stats -d $O/${EP}prof_$cfg -o run --output-format csv -- \
      python3 bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-parity
  fi
  if has pmc; then
    B="python3 bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-parity"
    step ${EP}pmc_${cfg}_fetch 200 rocprofv3 --kernel-include-regex $K --pmc FETCH_SIZE -d $O/${EP}pmc_${cfg}_fetch -o run --output-format csv -- $B
    step ${EP}pmc_${cfg}_write 200 rocprofv3 --kernel-include-regex $K --pmc WRITE_SIZE -d $O/${EP}pmc_${cfg}_write -o run --output-format csv -- $B
    step ${EP}pmc_${cfg}_sq 200 rocprofv3 --kernel-include-regex $K --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU \
      SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $O/${EP}pmc_${cfg}_sq -o run --output-format csv -- $B
  fi
  if has e2e; then
    case $cfg in
      config2) step e2e_$cfg 300 python3 tools/e2e_bench.py --config $cfg --records 262144 --chunk 8192 ;;
      config3) step e2e_$cfg 300 python3 tools/e2e_bench.py --config $cfg --records 1048576 --chunk 65536 ;;
    esac
  fi
done
