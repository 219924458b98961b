"""Diagnostics: host-side time of every library call of a B = 544 training
step (per-step kernels, side-stream gate on) after full-shape steps of the
bench configurations -- finds a host call that blocks on the device while the
side-stream gate spins."""
import os, sys, time, torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, REPO + "/seq2seq_abcd-vae_amd")
import bench
from modules import engine, noise, _native as N

lib = N.lib()
log = []


class Proxy:
    def __getattr__(self, name):
        f = getattr(lib, name)
        if not callable(f):
            return f

        def g(*a):
            t0 = time.perf_counter()
            r = f(*a)
            log.append((name, (time.perf_counter() - t0) * 1e3))
            return r
        return g


pre = [("c2", 512), ("c4", 512), ("c5", 128), ("c5gru", 128), ("c5", 512), ("c5gru", 512)]
if len(sys.argv) > 1:
    pre = pre[:int(sys.argv[1])]
for name, B in pre:
    cfg = dict(bench.CONFIGS[name], B=B)
    batch = bench.make_batch(cfg, 1, "cpu")
    step = bench.build(cfg, "cuda")
    step.forward_backward(batch["data"].cuda(), batch["batch_sizes"], batch["is_offset"].cuda(),
                          batch["speakers"].cuda(), cfg["N"])
    torch.cuda.synchronize()
    print("pre", name, B, flush=True)
N.lib = lambda: Proxy()
engine.N.lib = N.lib
cfg = dict(bench.CONFIGS["c2"], B=544, tmin=12, tmax=24)
batch = bench.make_batch(cfg, 77, "cpu")
step = bench.build(cfg, "cuda")
args = (batch["data"].cuda(), batch["batch_sizes"], batch["is_offset"].cuda(), batch["speakers"].cuda(), cfg["N"])
for k in range(4):
    log.clear()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step.forward_backward(*args)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("call %d: host %.2f ms, +sync %.2f ms; calls > 1 ms: %s" % (
        k, (t1 - t0) * 1e3, (t2 - t1) * 1e3, [(n, round(d, 2)) for n, d in log if d > 1.0]), flush=True)
