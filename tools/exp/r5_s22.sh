#!/bin/bash
# Round 5, session 22: the ragged long class at 8 lanes per record in the table-free
# engine: parity of both engines, then
# configs 2 / G / 4 / 5 of both, and the bitsliced engine with temporal loads too.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-r5s22}
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
step pytest_par 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread
step pytest_bs_total 500 env BSSL_AMD_GCM_MODE=bs python -u -m pytest tests/test_bs16_total.py -x -q --timeout 200 --timeout-method thread
for cfg in config2 configG config4 config5; do
  step t_$cfg 200 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline
  step bs_$cfg 200 env BSSL_AMD_GCM_MODE=bs python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline
done
