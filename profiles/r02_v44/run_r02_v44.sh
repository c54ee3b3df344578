set -o pipefail
# Longer progress-poll naps (r02_v42: always 8 x 64 cycles was best, -1.5 %):
# pc = 8, pd = 16, pe = 32 (x 64 cycles) on every poll.
D=gpurun_out/r02_v44
mkdir -p $D
export TMPDIR=/tmp
V=$PWD/svscope_amd/lib/variants
p() { SVS_LIB_PATH=$V/libsvscope_hip_$1.so timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_$1$2.log 2>&1; }
p pc 1 && p pd 1 && p pe 1 && p pc 2 && p pd 2 && p pe 2
