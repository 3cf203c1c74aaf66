# One gpurun attempt of a call script after an optional pause (no retry loop):
# usage: bash scripts/try_gpu.sh <pause-seconds> <call-script> <outfile>
sleep $1
/usr/local/graft/bin/gpurun --timeout 1200 -- "bash $2" > $3 2>&1
echo "exit $?" >> $3
