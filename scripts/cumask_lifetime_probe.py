"""Which lifetime orders of CU-masked external streams vs tensors allocated on them are
safe? Each case runs in its own process; prints the exit code."""
import subprocess
import sys

CASE = r'''
import sys, torch
sys.path.insert(0, ".")
from omldm_amd.ops import native
lib = native.hip()
dev = torch.device("cuda", 0)
torch.cuda.init()
raw = lib.omldm_stream_create_cumask_ex(16, 1, 1)
s = torch.cuda.ExternalStream(raw, device=dev)
with torch.cuda.stream(s):
    x = torch.ones(1 << 20, device=dev) * 2
    y = x + 1
torch.cuda.synchronize()
case = sys.argv[1]
if case == "free_then_destroy":
    del x, y
    torch.cuda.synchronize()
    lib.omldm_stream_destroy(raw)
elif case == "destroy_then_free":
    torch.cuda.synchronize()
    lib.omldm_stream_destroy(raw)
    del x, y
    torch.cuda.empty_cache()
elif case == "destroy_keep_alive":
    torch.cuda.synchronize()
    lib.omldm_stream_destroy(raw)
elif case == "never_destroy":
    pass
elif case == "free_emptycache_destroy":
    del x, y
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    lib.omldm_stream_destroy(raw)
print("done", case, flush=True)
'''

for case in ("free_then_destroy", "destroy_then_free", "destroy_keep_alive", "never_destroy",
             "free_emptycache_destroy"):
    r = subprocess.run([sys.executable, "-c", CASE, case], capture_output=True, text=True,
                       timeout=120)
    print(f"{case:26s} rc={r.returncode} {r.stdout.strip()[-40:]}", flush=True)
