set -x
nproc; cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null; taskset -p $$
ls /sys/devices/system/node/ | head; 
python - <<'PY'
import torch, os
n = torch.cuda.device_count(); print("devices", n)
for i in range(n):
    p = torch.cuda.get_device_properties(i)
    print(i, p.name, {k: getattr(p, k, None) for k in ("pci_bus_id","pci_device_id","pci_domain_id","gcnArchName","multi_processor_count")})
PY
for d in /sys/class/drm/card*/device; do echo $d $(cat $d/numa_node 2>/dev/null) $(readlink -f $d) $(cat $d/local_cpulist 2>/dev/null) $(cat $d/current_link_speed $d/current_link_width 2>/dev/null); done
rocm-smi --showtoponuma 2>&1 | tail -20
rocm-smi --showbus 2>&1 | tail -10
