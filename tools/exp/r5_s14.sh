#!/bin/bash
# Round 5, session 14: where the output pass's memory cost comes from -- same-box
# config 2 lines of the product build against output passes without the
# plaintext loads, without the ciphertext stores, with temporal (non-nt)
# stores, with temporal loads; phase clocks of the product build.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-r5s14}
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
export BSSL_AMD_GCM_MODE=bs
L=boringssl_amd/csrc/build
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity --config config2"
step prof 200 env BSSL_AMD_LIB=$L/ab_prof/libbssl_amd.so python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --config config2
grep bs_prof $O/prof.log | tail -1
for v in base noload nostore plainst plainld base; do
  if [ $v = base ]; then step c2_$v 200 $B; else step c2_$v 200 env BSSL_AMD_LIB=$L/ab_$v/libbssl_amd.so $B; fi
done
