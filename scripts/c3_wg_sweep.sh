O="--no-cpu --no-handoff --mapping-steps 0 --fleet-streams 0 --loop-scans 0"
for g in 16 24 32 48; do
  LEGO_ODOM_WORKGROUPS=$g timeout -k 10 120 python bench.py $O --dense-scans 0 --sensor HDL-64E --seed 2 --stream-len 200 --batch 20 --steps 8 --warmup 2 > gpurun_out/c3g$g.log 2>&1 || exit 1
done
timeout -k 10 200 python bench.py $O --dense-scans 200 --stream-len 100 --steps 1 --warmup 0 > gpurun_out/c3dense.log 2>&1
