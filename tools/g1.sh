set -o pipefail
mkdir -p gpurun_out/g5
export TMPDIR=/tmp
for w in 0 64 1024; do
SG_LIT_SHARE_W=$w SG_LIT_DEBUG=8 timeout -k 10 120 python -u tools/c4_probe.py 1000000 2>&1 | grep -m1 re_prefilter
SG_LIT_SHARE_W=$w timeout -k 10 120 python -u tools/c4_probe.py 4000000 > gpurun_out/g5/c4_$w.log 2>&1 || exit 1; echo "w $w"; tail -1 gpurun_out/g5/c4_$w.log
SG_LIT_SHARE_W=$w timeout -k 10 120 python -u tools/c3_probe.py > gpurun_out/g5/c3_$w.log 2>&1 || exit 1; tail -1 gpurun_out/g5/c3_$w.log
done
