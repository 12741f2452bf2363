set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=$PWD/boringssl_amd/csrc/build
BSSL_AMD_LIB=$B/ab_pfst/libbssl_amd.so timeout -k 10 300 python bench.py --config configG --steps 1 --warmup 0 --no-cpu-baseline --no-parity > gpurun_out/s22_stamps_G.txt 2>&1 || exit 1
grep -h "stamps block 0" gpurun_out/s22_stamps_G.txt | head -8
SPECS="configG:ab_pf config2:ab_pf config4:ab_pf" REPS="1 2" timeout -k 10 800 bash tools/exp/ab_session.sh > gpurun_out/s22_ab.txt 2>&1; cat gpurun_out/s22_ab.txt
