for gp in 64 128 256 512; do
  for tc in 1536 3072 6144; do
    YOUTH_ICP_TARGET_CHUNKS=$tc timeout -k 10 120 python3 bench.py --global-pairs $gp --steps 30 --warmup 5 --no-cpu-baseline --no-host-io --no-legs --no-viewer > gpurun_out/sw_${gp}_${tc}.json 2>/dev/null || exit 1
    python3 -c "
import json;d=json.load(open('gpurun_out/sw_${gp}_${tc}.json'))
print('pairs ${gp} chunks ${tc}: %.0f aligns/s  k_icp %.1f us  prep %.1f us  step %.1f us  sched %s' % (d['value'], d['roofline']['avg_launch_ms']*1e3, d['kernel_ms_per_step']['k_prep']*1e3, d['ms_per_step']*1e3, d['sched_last_step']))"
  done
done
