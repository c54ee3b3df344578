set -o pipefail
D=gpurun_out/r02_v15
mkdir -p $D
export TMPDIR=/tmp
SVS_POA_DEBUG=1 timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_narrow_dbg.log 2>&1 && \
SVS_POA_WIDE=1 SVS_POA_DEBUG=1 timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_wide_dbg.log 2>&1 && \
SVS_POA_WIDE=1 SVS_POA_WPJ=2 timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_wide_wpj2.log 2>&1 && \
SVS_POA_WIDE=1 SVS_LIB_PATH=$PWD/svscope_amd/lib/variants/libsvscope_hip_wocc3.so timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_wide_occ3.log 2>&1 && \
SVS_POA_WIDE=1 SVS_LIB_PATH=$PWD/svscope_amd/lib/variants/libsvscope_hip_wocc5.so timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_wide_occ5.log 2>&1
