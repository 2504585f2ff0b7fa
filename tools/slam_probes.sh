#!/bin/bash
# Round-5 probes of the drop-in's ingest path, one
# subcommand each; run on the GPU box through `tools/gpu_call.sh TAG
# sh:tools/slam_probes.sh` with PROBE=<name> in the environment, or directly.
# Output under gpurun_out/slamprobe_<name>/; DESIGN.md §6 quotes the results
# kept in profiles/r05/.
#   copy_paths  examples/slam_rate (20 backlogged passes, event trace) with the
#               default k_pull_frames copy and with YOUTH_ICP_TRACK_COPY=sdma
#   pull_sweep  the pull's free-CU reservation and workgroups per frame
#   trace       one slam_rate run under rocprofv3 --kernel-trace
#               --memory-copy-trace, the per-pass summary and the copies'
#               overlap with k_icp_coop (tools/copy_overlap.py)
#   sdma        tools/sdma_probe: the tracker's copy pattern in a plain HIP
#               program (does any hipMemcpyAsync enqueue block > 1 ms?)
#   library     tools/trk_stall_probe.py: the tracker driven from one thread
#   runtime_log slam_rate with AMD_LOG_LEVEL=4 (the HIP runtime's own log)
#   live        slam_rate under rocprofv3 --kernel-trace with the event trace:
#               where a live frame's processSlamFrame -> pose time goes
#               (tools/slam_trace.py --live)
set -eo pipefail
export TMPDIR=/tmp
PROBE=${PROBE:-${1:-copy_paths}}
O=gpurun_out/slamprobe_$PROBE
mkdir -p $O
echo "host: $(nproc) cpus visible, loadavg $(cat /proc/loadavg)"

slam_rate_run() {  # label passes env...
  local label=$1 passes=$2
  shift 2
  env "$@" YOUTH_SLAM_TRACE=$O/events_$label.txt timeout -k 10 120 slam-rgbd_amd/slam_rate 300 $passes \
      > $O/slam_rate_$label.json 2> $O/slam_rate_$label.err
  python3 tools/slam_trace.py $O/events_$label.txt > $O/summary_$label.txt
  echo "== $label: $(python3 -c "import json;d=json.load(open('$O/slam_rate_$label.json'));print(d['value'], [round(v/1e3,1) for v in d['pass_values']], 'live', d['live_latency_us_median'])")"
  grep "slow submit" $O/summary_$label.txt || true
}

case $PROBE in
  live)
    YOUTH_SLAM_TRACE=$O/events_live.txt timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv \
        -d $O/kt_live -o kt -- slam-rgbd_amd/slam_rate 300 4 > $O/slam_rate_live.json 2> $O/slam_rate_live.err
    KT=$(find $O/kt_live -name '*kernel_trace.csv' -print -quit)
    python3 tools/slam_trace.py --live $O/events_live.txt.live $KT | tee $O/live_summary.txt
    YOUTH_SLAM_TRACE=$O/events_live_noprof.txt timeout -k 10 120 slam-rgbd_amd/slam_rate 300 4 \
        > $O/slam_rate_live_noprof.json 2> $O/slam_rate_live_noprof.err
    python3 tools/slam_trace.py --live $O/events_live_noprof.txt.live | tee $O/live_summary_noprof.txt ;;
  copy_paths)
    slam_rate_run pull 20
    slam_rate_run sdma 20 YOUTH_ICP_TRACK_COPY=sdma
    slam_rate_run pull_b 20
    slam_rate_run sdma_b 20 YOUTH_ICP_TRACK_COPY=sdma ;;
  pull_sweep)
    for r in 0 16 24 32; do
      for w in 2 4; do
        slam_rate_run r${r}w$w 12 YOUTH_ICP_PULL_RESERVE_CU=$r YOUTH_ICP_PULL_WG=$w
      done
    done
    slam_rate_run nolds 12 YOUTH_ICP_PULL_LDS=0 ;;
  trace)
    for cfg in "pull" "sdma YOUTH_ICP_TRACK_COPY=sdma"; do
      set -- $cfg
      label=$1
      shift
      env "$@" YOUTH_SLAM_TRACE=$O/events_$label.txt timeout -k 10 120 rocprofv3 --kernel-trace \
          --memory-copy-trace --output-format csv -d $O/kt_$label -o kt -- slam-rgbd_amd/slam_rate 300 6 \
          > $O/slam_rate_$label.json 2> $O/slam_rate_$label.err
      KT=$(find $O/kt_$label -name '*kernel_trace.csv' -print -quit)
      python3 tools/slam_trace.py $O/events_$label.txt $KT > $O/summary_$label.txt
      echo "== $label"
      grep "^pass\|slow submit" $O/summary_$label.txt
      python3 tools/copy_overlap.py $O/kt_$label
    done ;;
  sdma)
    timeout -k 10 60 tools/sdma_probe 2000 40 5
    timeout -k 10 60 tools/sdma_probe 2000 0 0 ;;
  library)
    for mode in reuse fresh fresh-thread; do
      echo "== $mode"
      timeout -k 10 120 python3 tools/trk_stall_probe.py 20 $mode
    done ;;
  runtime_log)
    AMD_LOG_LEVEL=4 YOUTH_SLAM_TRACE=$O/events.txt timeout -k 10 120 slam-rgbd_amd/slam_rate 300 4 \
        > $O/slam_rate.json 2> $O/hiplog.txt
    python3 tools/slam_trace.py $O/events.txt | grep "^pass\|slow submit" ;;
  *)
    echo "unknown probe $PROBE"
    exit 2 ;;
esac
