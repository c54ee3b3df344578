#!/bin/bash
# Strip-kernel clock profile (SVS_STRIP_PROF variant) of the MSA probe under
# several launch shapes.  tools/sprof_sweep.sh NAME 'label ENV=V ...' ...
set -o pipefail
N=${1:?name}; shift
D=gpurun_out/$N
mkdir -p $D
export TMPDIR=/tmp
for spec in "$@"; do
  set -- $spec
  label=$1; shift
  env SVS_STRIP_PROF=1 SVS_LIB_PATH=svscope_amd/lib/variants/libsvscope_hip_sprof.so "$@" timeout -k 10 200 python3 tools/poa_probe.py --windows 1024 > $D/p_$label.log 2>&1 || { tail -5 $D/p_$label.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$D/p_$label.log') if l.startswith('{')][-1]); p=d['strip_prof']; L=p['life_cyc']
print('$label', 'kernel_ms', round(d['kernel_ms']), 'waves', p['waves'], ' '.join('%s=%.3f' % (k[:-4], p[k]/L) for k in ('fetch_wait_cyc','ff_wait_cyc','ff_cyc','sweep_cyc','tb_cyc','end_barrier_cyc')), 'cyc/row %.0f' % (L/p['rows_computed']))"
done
