# PMC passes over tools/exp/modes.py (table, mix4, bs16): VALU/SALU cycles vs
# instructions of the T-table, mixed-role and bs16 kernels.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp N=262144
P="python3 tools/exp/modes.py table mix4 bs16"
timeout -s KILL 90 rocprofv3 --kernel-include-regex "gcm_(mix_)?kernel" --pmc SQ_INSTS_VALU SQ_INST_CYCLES_VALU SQ_INSTS_SALU SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc3 -o run --output-format csv -- $P > gpurun_out/pmc3.log 2>&1
