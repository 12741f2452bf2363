#!/bin/bash
# Round 5, session 19: non-temporal vs temporal record stores (config G's
# L = 4 T-table kernel fetches ~2x its record bytes by the calibrated count:
# half-line nt stores filled by read-modify-write?): same-box lines of both
# engines with temporal stores, and FETCH/WRITE of config G under each.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-r5s19}
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | head -1)" | tee -a $O/steps.log
  [ $rc -eq 0 ] || { tail -5 $O/$name.log; exit $rc; }
}
L=boringssl_amd/csrc/build
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity --config"
for cfg in configG config4 config2 config5; do
  step t_$cfg 200 $B $cfg
  step tplain_$cfg 200 env BSSL_AMD_LIB=$L/ab_tplain/libbssl_amd.so $B $cfg
done
for cfg in configG config2; do
  step bs_$cfg 200 env BSSL_AMD_GCM_MODE=bs $B $cfg
  step bsplain_$cfg 200 env BSSL_AMD_GCM_MODE=bs BSSL_AMD_LIB=$L/ab_bsplain/libbssl_amd.so $B $cfg
done
P="python3 bench.py --config configG --steps 2 --warmup 1 --no-cpu-baseline --no-parity"
for v in base tplain; do
  if [ $v = base ]; then E=""; else E="$L/ab_$v/libbssl_amd.so"; fi
  step pmcf_$v 120 env BSSL_AMD_LIB=${E:-boringssl_amd/libbssl_amd.so} rocprofv3 --kernel-include-regex gcm_kernel --pmc FETCH_SIZE -d $O/pmcf_$v -o run --output-format csv -- $P
  step pmcw_$v 120 env BSSL_AMD_LIB=${E:-boringssl_amd/libbssl_amd.so} rocprofv3 --kernel-include-regex gcm_kernel --pmc WRITE_SIZE -d $O/pmcw_$v -o run --output-format csv -- $P
done
