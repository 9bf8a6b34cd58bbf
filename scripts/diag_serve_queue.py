"""Does a kernel on the current stream wait behind the persistent serving wave?
For several stream choices for the wave and several numbers of pre-created streams."""
import sys, time, torch
sys.path.insert(0, ".")
from omldm_amd.api.batch import FeatureSpace
from omldm_amd.io.synthetic import synth_batch
from omldm_amd.ops import native
from omldm_amd.ops import serving as SV

dev = torch.device("cuda", 0)
sp = FeatureSpace(13, 0, 26, 1 << 16, field_aware=True)
w = torch.randn(sp.dim, device=dev).to(torch.bfloat16)
x = torch.zeros(1 << 20, device=dev)
keep = []
for variant in ("pool", "cumask", "high"):
    for extra in range(0, 6):
        for _ in range(extra):
            keep.append(torch.cuda.Stream(dev))
        srv = SV.PredictServer.__new__(SV.PredictServer)
        srv.lib = SV._lib(); srv.W = w.unsqueeze(0); srv.M, srv.dim = 1, sp.dim
        srv.dn, srv.dc, srv.bias, srv.cspan = sp.dn, sp.dc, True, sp.cat_span
        srv.mb = srv.lib.omldm_mailbox_alloc(); srv._raw_stream = None
        if variant == "pool":
            srv.stream = torch.cuda.Stream(dev)
        elif variant == "cumask":
            srv._raw_stream = native.hip().omldm_stream_create_cumask(0)
            srv.stream = torch.cuda.ExternalStream(srv._raw_stream, device=dev)
        else:
            srv.stream = torch.cuda.Stream(dev, priority=-1)
        import ctypes as C
        srv.out = (C.c_float * 1)()
        srv.start(lifetime_us=3_000_000)
        t = time.time()
        x.add_(1)
        torch.cuda.current_stream().synchronize()
        dt = time.time() - t
        srv.close()
        print(f"{variant:7s} extra={extra} current-stream op took {dt*1e3:9.2f} ms", flush=True)
