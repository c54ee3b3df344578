#!/bin/bash
# Same-box A/B of bench.py configurations (AB_STEPS timed steps, default 10; AB_WARMUP
# warm-up steps, default 2; no CPU baseline).
#   tools/ab_bench.sh NAME 'label1 ENV=V ...' 'label2 ENV=V ...' ...
# A label's environment may set SVS_LIB_PATH to a development variant
# (tools/build_variant.py).  Prints value, mean DP launch, DP kernel seconds and
# the oracle digest check per run.
set -o pipefail
N=${1:?name}; shift
D=gpurun_out/$N
mkdir -p $D
export TMPDIR=/tmp
for spec in "$@"; do
  set -- $spec
  label=$1; shift
  env "$@" timeout -k 10 240 python3 bench.py --steps ${AB_STEPS:-10} --warmup ${AB_WARMUP:-2} --cpu-sample 0 > $D/b_$label.json 2> $D/b_$label.err || { tail -20 $D/b_$label.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/b_$label.json')); b=d['breakdown']; print('$label', d['value'], 'busy', d['roofline']['frac'], 'wall', d['roofline']['frac_over_wall'], 'launch', d['roofline']['per_launch']['frac'], d['roofline']['per_launch']['mean_launch_ms'], round(b['poa_kernel_ms']/1e3, 2), b['poa_launches'], d['oracle_check']['match'], b.get('fold_kernel_ms'))"
done
