set -o pipefail
# Progress-poll nap schedule A/B on the MSA probe (SVS_POLL_N / S1 / S2:
# the first N polls sleep S1 x 64 cycles, later ones S2 x 64):
# cur = 8 / 1 / 4 (product), pa = 4 / 2 / 8, pb = 2 / 4 / 8, pc = 0 / - / 8.
D=gpurun_out/r02_v42
mkdir -p $D
export TMPDIR=/tmp
V=$PWD/svscope_amd/lib/variants
p() { SVS_LIB_PATH=$V/libsvscope_hip_$1.so timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_$1$2.log 2>&1; }
p cur 1 && p pa 1 && p pb 1 && p pc 1 && p cur 2 && p pa 2 && p pb 2 && p pc 2
