set -o pipefail
mkdir -p gpurun_out/r06_s2
export TMPDIR=/tmp
AB_STEPS=20 AB_WARMUP=5 bash tools/ab_bench.sh r06_s2 'base SVS_POA_FOLD_WORKERS=0' 'w256p0 SVS_POA_FOLD_WORKERS=256 SVS_POA_FOLD_PRIO=0' 'w128p0 SVS_POA_FOLD_WORKERS=128 SVS_POA_FOLD_PRIO=0' 'w64p3 SVS_POA_FOLD_WORKERS=64 SVS_POA_FOLD_PRIO=3' 'w128p1 SVS_POA_FOLD_WORKERS=128 SVS_POA_FOLD_PRIO=1' 'base2 SVS_POA_FOLD_WORKERS=0'
for f in gpurun_out/r06_s2/b_*.json; do python3 -c "import json;d=json.load(open('$f'));b=d['breakdown'];print('$f', b['dp_end_to_launch_done_ms'], b['poa_launches'], round(b['dp_end_to_launch_done_ms']/b['poa_launches'],2), b['em_kernel_s'], d['roofline']['busy_ms'])"; done
