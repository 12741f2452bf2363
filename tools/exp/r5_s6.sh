#!/bin/bash
# Round 5, session 6: table-free engine with full-chunk asm variants and
# L = 2 for short records: parity, then both engines on configs 2, G, 4, 5.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-r5s6}
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a $O/steps.log
  tail -1 "$O/$name.log" | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
}
step pytest_bs 400 python -u -m pytest tests/test_gpu_parity.py -k "bitsliced or mix_kernel" -x -q --timeout 120 --timeout-method thread
step pytest_bs_total 500 python -u -m pytest tests/test_bs16_total.py -x -q --timeout 200 --timeout-method thread
for cfg in config2 configG config4 config5; do
  step ${cfg}_table 200 env BSSL_AMD_GCM_MODE=table python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline
  step ${cfg}_bs 200 env BSSL_AMD_GCM_MODE=bs python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline
done
