#!/bin/bash
# Round 5, session 23: table-free engine with its record start and end at
# s_setprio 1 / 2 (latency-bound phases, as the output pass): same-box lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-r5s23}
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | head -1) $(grep -o '"parity": "[a-z_]*' $O/$name.log | head -1)" | tee -a $O/steps.log
  [ $rc -eq 0 ] || { tail -5 $O/$name.log; exit $rc; }
}
export BSSL_AMD_GCM_MODE=bs
L=boringssl_amd/csrc/build
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --config"
for cfg in config2 configG config5 config4; do
  step base_$cfg 200 $B $cfg
  step edge1_$cfg 200 env BSSL_AMD_LIB=$L/ab_edge1/libbssl_amd.so $B $cfg
  step edge2_$cfg 200 env BSSL_AMD_LIB=$L/ab_edge2/libbssl_amd.so $B $cfg
done
