set -o pipefail
D=gpurun_out/r02_v8
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_em_gpu.py -x -v --timeout 240 --timeout-method thread > $D/pytest_em.log 2>&1 && \
timeout -k 10 300 python -u tools/em_probe.py --windows 1024 > $D/em_probe_gather.log 2>&1 && \
SVS_EM_MFMA=1 timeout -k 10 300 python -u tools/em_probe.py --windows 1024 > $D/em_probe_mfma.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $D/pmc_gather -o run -- python3 tools/em_probe.py --windows 256 > $D/pmc_gather.log 2>&1 && \
SVS_EM_MFMA=1 timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $D/pmc_mfma -o run -- python3 tools/em_probe.py --windows 256 > $D/pmc_mfma.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt_gather -o run -- python3 tools/em_probe.py --windows 1024 > $D/kt_gather.log 2>&1 && \
SVS_EM_MFMA=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt_mfma -o run -- python3 tools/em_probe.py --windows 1024 > $D/kt_mfma.log 2>&1
