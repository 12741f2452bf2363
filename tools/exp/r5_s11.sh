#!/bin/bash
# Round 5, session 11: E_K(J0) flags one per 128-byte line, polled with RMW
# atomics: parity, phase clocks (configs 2 and G), configs 2 / G / 4 / 5 of
# both engines, the output pass at s_setprio 2 and the ablations (1 no GHASH,
# 3 no GHASH and no record I/O, 4 no output pass) on config 2.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-r5s11}
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | head -1) $(grep -o 'ref_digest_[a-z]*' $O/$name.log | head -1)" | tee -a $O/steps.log
  [ $rc -eq 0 ] || { tail -5 $O/$name.log; exit $rc; }
}
export BSSL_AMD_GCM_MODE=bs
step pytest_bs 400 python -u -m pytest tests/test_gpu_parity.py -k "bitsliced or mix_kernel" -x -q --timeout 120 --timeout-method thread
step pytest_bs_total 500 python -u -m pytest tests/test_bs16_total.py -x -q --timeout 200 --timeout-method thread
L=boringssl_amd/csrc/build
step prof_c2 200 env BSSL_AMD_LIB=$L/ab_prof/libbssl_amd.so python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --config config2
grep bs_prof $O/prof_c2.log | tail -1
step prof_cG 200 env BSSL_AMD_LIB=$L/ab_prof/libbssl_amd.so python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --config configG
grep bs_prof $O/prof_cG.log | tail -1
for cfg in config2 configG config4 config5; do
  step ${cfg}_table 200 env BSSL_AMD_GCM_MODE=table python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline
  step ${cfg}_bs 200 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline
  step ${cfg}_prio2 200 env BSSL_AMD_LIB=$L/ab_prio2/libbssl_amd.so python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-parity
done
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity --config config2"
for n in 1 3 4; do step c2_abl$n 200 env BSSL_AMD_LIB=$L/ab_abl$n/libbssl_amd.so $B; done
