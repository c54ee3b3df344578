# probe A/B: kernel ms of the MSA probe (1024 config-3 windows)
D=gpurun_out/$1; shift
mkdir -p $D
for spec in "$@"; do
  set -- $spec; label=$1; shift
  env "$@" timeout -k 10 200 python3 tools/poa_probe.py --windows 1024 > $D/p_$label.log 2>&1 || { tail -5 $D/p_$label.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$D/p_$label.log') if l.startswith('{')][-1])
print('$label', 'kernel_ms', round(d['kernel_ms'],1), 'wall_ms', round(d['wall_ms']), 'launches', d['launches'])"
done
