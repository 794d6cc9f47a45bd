set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_FLAT SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU --kernel-trace --stats -d $R/gpurun_out/pmc_codec2 -o run -- python3 scripts/exp/codec_only.py > gpurun_out/pmc_codec2.log 2>&1; echo rc=$?; tail -3 gpurun_out/pmc_codec2.log; ls -R gpurun_out/pmc_codec2 | head
