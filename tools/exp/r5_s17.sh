#!/bin/bash
# Round 5, session 17: per-group E_K(J0) timing (production start/end, first
# consumer arrival, first claim) of the table-free engine on config 2.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-r5s17}
mkdir -p $O
export BSSL_AMD_GCM_MODE=bs
timeout -k 10 200 env BSSL_AMD_LIB=boringssl_amd/csrc/build/ab_prof/libbssl_amd.so python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --config config2 > $O/prof_config2.log 2>&1
rc=$?
grep "bs_grp groups\|bs_prof" $O/prof_config2.log | tail -4
grep "bs_grp late" $O/prof_config2.log | tail -20
exit $rc
