#!/bin/bash
# Round 5, session 16: where the units that wait for their E_K(J0) sit in the
# batch (phase-clock build with position buckets), configs 2 and G.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-r5s16}
mkdir -p $O
export BSSL_AMD_GCM_MODE=bs
L=boringssl_amd/csrc/build
for cfg in config2 configG; do
  timeout -k 10 200 env BSSL_AMD_LIB=$L/ab_prof/libbssl_amd.so python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --config $cfg > $O/prof_$cfg.log 2>&1 || exit 1
  grep bs_prof $O/prof_$cfg.log | tail -2
done
