# round 5: is the fast/slow launch mode of a process (one-node graph replay ~2.5 vs ~10 us of host
# time, gpu_r5_launch_var.sh / gpu_r5_launch_aslr.sh) set by the CPU it runs on?  The probe pinned to
# the first CPU of every L3 domain (CCD), twice each.
set -o pipefail
O=${OUT:-gpurun_out/r5lc}
mkdir -p $O
export TMPDIR=/tmp
CPUS=$(python - <<'PY'
import glob, os
allowed = os.sched_getaffinity(0)
doms = {}
for f in glob.glob("/sys/devices/system/cpu/cpu[0-9]*/cache/index3/shared_cpu_list"):
    cpu = int(f.split("/")[5][3:])
    if cpu in allowed:
        doms.setdefault(open(f).read().strip(), []).append(cpu)
print(" ".join(str(min(v)) for v in sorted(doms.values(), key=min)))
PY
)
echo "L3 domains (first cpu each): $CPUS" | tee $O/ccd.txt
for rep in 1 2; do
  for c in $CPUS; do
    timeout -k 10 60 python scripts/graph_launch_probe.py --cpu $c > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
    grep launch-probe $O/p.log | tee -a $O/ccd.txt
  done
done
echo done
