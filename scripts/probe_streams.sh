set -o pipefail
mkdir -p gpurun_out
export LEGO_ODOM_PLAIN_LAUNCH=1
for q in 4 16; do
 for g in 48 16 4 1; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python scripts/streams_probe.py --streams 1,4,5,8,16,32,64 --workgroups $g --stream-len 200 --batch 50 --steps 4 > gpurun_out/probe_q${q}_g${g}.log 2>&1 || { echo fail q$q g$g; tail -5 gpurun_out/probe_q${q}_g${g}.log; exit 1; }
  echo "q=$q"; grep streams gpurun_out/probe_q${q}_g${g}.log
 done
done
