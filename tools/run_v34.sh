set -o pipefail
mkdir -p gpurun_out
export SVS_LIB_PATH=$PWD/svscope_amd/lib/variants/libsvscope_hip_prof.so SVS_STRIP_PROF=1
timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > gpurun_out/v34_prof.log 2>&1 && \
SVS_POA_PRUNE=0 timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > gpurun_out/v34_prof_noprune.log 2>&1
