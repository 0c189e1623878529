#!/bin/bash
# The blocking export's slow calls (pieces arriving ~5x slower over PCIe): which host side
# drives them.  Prints the box's NUMA layout and the GPU's node, then tools/blocking_seq.py
# (one-context C3 calls only) as is, with the transfers alone (no scatter: debug bit 22), and
# with the whole process on the GPU's node / on another node (taskset, before HIP starts).
# Usage (on the box): bash tools/blocking_numa.sh TAG
set -o pipefail
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p $OUT
for n in /sys/devices/system/node/node*; do echo "$(basename $n): $(cat $n/cpulist)"; done | tee $OUT/numa.txt
GN=$(cat /sys/class/drm/card*/device/numa_node 2>/dev/null | sort -u | tr '\n' ' ')
echo "gpu numa_node(s): $GN; allowed: $(grep Cpus_allowed_list /proc/self/status)" | tee -a $OUT/numa.txt
G=$(echo $GN | awk '{print $1}'); [ "$G" = "-1" ] && G=0
GC=$(cat /sys/devices/system/node/node$G/cpulist | cut -d, -f1)
OC=$(for n in /sys/devices/system/node/node*; do [ "$(basename $n)" != "node$G" ] && cat $n/cpulist && break; done | cut -d, -f1)
pick() { python3 -c "import os,sys; a=sorted(os.sched_getaffinity(0)); r=sys.argv[1]; lo,hi=map(int,r.split('-')) if '-' in r else (int(r),int(r)); s=[c for c in a if lo<=c<=hi][:16]; print(','.join(map(str,s)))" "$1"; }
GCP=$(pick $GC); OCP=$(pick ${OC:-0})
echo "gpu-node cpus: $GCP; other-node cpus: $OCP" | tee -a $OUT/numa.txt
run() { echo "== $1"; shift; env "$@" timeout -k 10 200 python3 -u tools/blocking_seq.py > $OUT/$N.txt 2> $OUT/$N.trace || { tail -3 $OUT/$N.trace; return 1; }; cut -c1-70 $OUT/$N.txt; }
for r in 1 2; do
  N=def_$r run "default $r" CONFIGS=C3 GROUP=0 REPS=24 || exit 1
  N=noscat_$r run "no scatter $r" CONFIGS=C3 GROUP=0 REPS=24 DEBUG=4194304 || exit 1
  if [ -n "$GCP" ]; then N=gnode_$r; echo "== gpu node $r"; CONFIGS=C3 GROUP=0 REPS=24 timeout -k 10 200 taskset -c $GCP python3 -u tools/blocking_seq.py > $OUT/$N.txt 2> $OUT/$N.trace || exit 1; cut -c1-70 $OUT/$N.txt; fi
  if [ -n "$OCP" ] && [ "$OCP" != "$GCP" ]; then N=onode_$r; echo "== other node $r"; CONFIGS=C3 GROUP=0 REPS=24 timeout -k 10 200 taskset -c $OCP python3 -u tools/blocking_seq.py > $OUT/$N.txt 2> $OUT/$N.trace || exit 1; cut -c1-70 $OUT/$N.txt; fi
done
