set -o pipefail
D=gpurun_out/r03_v13
mkdir -p $D
export TMPDIR=/tmp
SVS_POA_FOLD_TIMES=1 timeout -k 10 200 python3 bench.py --steps 4 --warmup 1 --cpu-sample 0 > $D/b_ft.json 2> $D/b_ft.err
rc=$?
grep "fold times" $D/b_ft.err
exit $rc
