# round 5: is the graph_module loop's process-to-process host variance CPU placement?  The GPU's
# PCI address -> NUMA node -> local CPUs, then the per-call breakdown pinned to a GPU-local core,
# a remote core, and unpinned.
set -o pipefail
O=${OUT:-gpurun_out/r5v}
mkdir -p $O
export TMPDIR=/tmp
python - > $O/numa.txt <<'PY'
import os, torch
p = torch.cuda.get_device_properties(0)
bus = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
d = f"/sys/bus/pci/devices/{bus}"
node = open(d + "/numa_node").read().strip() if os.path.exists(d) else "?"
local = open(d + "/local_cpulist").read().strip() if os.path.exists(d) else "?"
allowed = sorted(os.sched_getaffinity(0))
print("bus", bus, "node", node, "local", local)
print("allowed", len(allowed), allowed[:8], "...", allowed[-8:])
print("nodes", sorted(os.listdir("/sys/devices/system/node")))
for n in sorted(x for x in os.listdir("/sys/devices/system/node") if x.startswith("node")):
    print(n, open(f"/sys/devices/system/node/{n}/cpulist").read().strip())
PY
cat $O/numa.txt
LOCAL=$(python - <<'PY'
import os
t = open("gpurun_out/r5v/numa.txt").read().split()
local = t[t.index("local") + 1]
allowed = os.sched_getaffinity(0)
cpus = []
for part in local.split(","):
    a, _, b = part.partition("-")
    cpus += range(int(a), int(b or a) + 1)
ok = [c for c in cpus if c in allowed]
print(ok[len(ok) // 2] if ok else sorted(allowed)[0])
PY
)
REMOTE=$(python - <<'PY'
import os
t = open("gpurun_out/r5v/numa.txt").read().split()
local = t[t.index("local") + 1]
cpus = set()
for part in local.split(","):
    a, _, b = part.partition("-")
    cpus |= set(range(int(a), int(b or a) + 1))
ok = sorted(c for c in os.sched_getaffinity(0) if c not in cpus)
print(ok[len(ok) // 2] if ok else -1)
PY
)
echo "local core $LOCAL remote core $REMOTE"
for rep in 1 2 3; do
  for mode in local remote none; do
    case $mode in local) pre="taskset -c $LOCAL";; remote) [ "$REMOTE" = -1 ] && continue; pre="taskset -c $REMOTE";; none) pre="";; esac
    timeout -k 10 120 $pre python scripts/engine_step_breakdown.py --steps 3000 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
    echo "$mode $(grep breakdown $O/b.log)" | tee -a $O/gm_numa.txt
  done
done
echo done
