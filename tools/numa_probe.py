import os, torch, glob
p = torch.cuda.get_device_properties(0)
print({k: getattr(p, k) for k in dir(p) if 'pci' in k})
print("affinity", sorted(os.sched_getaffinity(0))[:8], len(os.sched_getaffinity(0)))
for d in glob.glob('/sys/bus/pci/devices/*'):
    try:
        cls = open(d + '/class').read().strip()
    except Exception:
        continue
    if cls.startswith('0x0380') or cls.startswith('0x1200'):
        print(d, cls, open(d + '/numa_node').read().strip(), open(d + '/local_cpulist').read().strip())
print(open('/sys/devices/system/node/online').read())
