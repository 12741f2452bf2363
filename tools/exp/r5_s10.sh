#!/bin/bash
# Round 5, session 10: table-free engine -- phase clocks with the record-end
# E_K(J0) wait split (flag poll / loads), then same-box config 2 lines of the
# product build against the output pass at s_setprio 2 and with (D, K) =
# (2, 4) / (1, 5) loads / GHASH lookups in flight; key-setup costs.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-r5s10}
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
step keysetup 100 python -u tools/keysetup_bench.py
L=boringssl_amd/csrc/build
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity --config"
step prof_c2 200 env BSSL_AMD_LIB=$L/ab_prof/libbssl_amd.so python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --config config2
grep bs_prof $O/prof_c2.log | tail -1
step prof_cG 200 env BSSL_AMD_LIB=$L/ab_prof/libbssl_amd.so python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --config configG
grep bs_prof $O/prof_cG.log | tail -1
for v in base prio2 dk24 dk15 base; do
  if [ $v = base ]; then step c2_$v 200 $B config2; else step c2_$v 200 env BSSL_AMD_LIB=$L/ab_$v/libbssl_amd.so $B config2; fi
done
step cG_base 200 $B configG
step cG_prio2 200 env BSSL_AMD_LIB=$L/ab_prio2/libbssl_amd.so $B configG
