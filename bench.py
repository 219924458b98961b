#!/usr/bin/env python3
"""Throughput of the ABCD-VAE training step (ABCD-VAE/learning.py:147-163) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c4|c5]

Metric (BASELINE.json): segments/sec/node for a full training step
(encoder -> sampler -> KL -> decoder -> loss -> backward -> all-reduce ->
clip -> SGD), weak scaling: b = 512 segments per GPU per step.  Workload
`c2` (default) is BASELINE.json configs[1]: synthetic segments, lengths
U{50..200} with the longest of each batch forced to 200 frames, 129 FFT bins,
K = 128, hidden 256, bi-LSTM encoder, self-feedback LSTM decoder, Gumbel
sampling on, N = 10,000.  Inputs are resident in HBM before the timed region;
noise is drawn in-kernel (Philox).

Besides the one JSON line the driver reads, it reports
  roofline     -- FP32-MFMA roofline of the dominant kernel family, timed live
                  with HIP events;
  cpu_baseline -- the CPU oracle (oracle/abcd_oracle.py, a torch-CPU
                  restatement of the reference step) timed on a bounded sample
                  on this host (rank 0, N = 1 only).
For N > 1 the driver launches it under torch.distributed.run (one rank per
GPU, RCCL, WORLD_SIZE set).  Run by hand as ``bench.py --gpus N`` without a
WORLD_SIZE, the process starts that same launcher as a CHILD (N fresh worker
processes; this parent never touches the GPU) and exits with its code.
"""
import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "seq2seq_abcd-vae_amd"))

PEAK_FP32_MFMA_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix 157.3 TF (dense, spec)

CONFIGS = {
    "c2": dict(workload="abcd-lstm synthetic 10k segments, T_max=200, F=129, K=128, h=256, b=512/GPU",
               F=129, H=256, Hm=256, D=256, K=128, rnn="LSTM", plain=False, tmin=50, tmax=200, B=512, N=10000,
               spk=0, sdim=None),
    "c4": dict(workload="plain gaussian-vae lstm, T_max=200, F=129, f=16, h=256, b=512/GPU",
               F=129, H=256, Hm=256, D=16, K=0, rnn="LSTM", plain=True, tmin=50, tmax=200, B=512, N=10000,
               spk=0, sdim=None),
    "c5": dict(workload="abcd-lstm stress K=1024, speaker_dim=256 (16 spk), T_max=512, F=129, h=256, b=512/GPU",
               F=129, H=256, Hm=256, D=256, K=1024, rnn="LSTM", plain=False, tmin=128, tmax=512, B=512,
               N=10000, spk=16, sdim=256),
    "c5gru": dict(workload="abcd-gru stress K=1024, speaker_dim=256 (16 spk), T_max=512, F=129, h=256, b=512/GPU",
                  F=129, H=256, Hm=256, D=256, K=1024, rnn="GRU", plain=False, tmin=128, tmax=512, B=512,
                  N=10000, spk=16, sdim=256),
}


def flops_per_step(cfg, L, B):
    """Algorithmic GEMM FLOPs of one training step: 3 x forward."""
    F, H, Hm, D, K = cfg["F"], cfg["H"], cfg["Hm"], cfg["D"], cfg["K"]
    G = 4 if cfg["rnn"] == "LSTM" else 3
    enc = 2 * 2 * (F + H) * G * H
    dec = 2 * (F + H) * G * H + 2 * (2 * H * Hm + 2 * Hm * F) + (2 * H * Hm + 2 * Hm)
    E = 4 * H if cfg["rnn"] == "LSTM" else 2 * H
    Hdec = 2 * H if cfg["rnn"] == "LSTM" else H
    S = cfg["sdim"] or 0
    if cfg["plain"]:
        seg = 2 * (2 * E * Hm + 2 * Hm * D) + 2 * (D + S) * Hdec
    else:
        seg = 2 * E * Hm + 2 * Hm * D + 2 * D * K + 2 * K * D + 2 * (D + S) * Hdec
    return 3 * ((enc + dec) * L + seg * B)


# timing ids of the persistent-kernel roles (abcd_timing_*); the kernel each
# role dispatched is read back from the library (abcd_dispatch_name)
KERNELS = {1: "enc_fwd", 2: "enc_bwd", 3: "dec_fwd", 4: "dec_bwd"}


def kernel_flops_per_frame(cfg, kid):
    """Algorithmic FLOPs per packed frame of one persistent kernel (unpadded
    dims, 2 per multiply-add).  Encoder: the recurrent products of both
    directions (the input projection is a separate GEMM).  Decoder forward:
    [x|h] W^T of the cell + the two emission MLP layers; decoder backward the
    transposed products of the same three layers."""
    F, H, Hm = cfg["F"], cfg["H"], cfg["Hm"]
    G = 4 if cfg["rnn"] == "LSTM" else 3
    if kid in (1, 2):
        return 2 * 2 * H * G * H
    return 2 * (F + H) * G * H + 2 * H * 2 * Hm + 2 * 2 * Hm * F


def make_batch(cfg, seed, device):
    g = torch.Generator().manual_seed(seed)
    B, tmin, tmax = cfg["B"], cfg["tmin"], cfg["tmax"]
    lens = torch.randint(tmin, tmax + 1, (B,), generator=g)
    lens[0] = tmax
    lens, _ = torch.sort(lens, descending=True)
    T = int(lens[0])
    bs = torch.tensor([int((lens > t).sum()) for t in range(T)], dtype=torch.int64)
    L = int(bs.sum())
    data = torch.randn(L, cfg["F"], generator=g)
    is_off = torch.zeros(L)
    off = 0
    for t in range(T):
        n = int(bs[t])
        ends = (lens[:n] == t + 1).nonzero().flatten()
        is_off[off + ends] = 1.0
        off += n
    spk = torch.randint(0, max(cfg["spk"], 1), (B,), generator=g)
    return dict(data=data.to(device), batch_sizes=bs, is_offset=is_off.to(device), speakers=spk.to(device),
                lengths=lens, L=L, T=T)


def build(cfg, device):
    from modules import model as M, engine
    torch.manual_seed(1111)
    enc = M.RNN_Variational_Encoder(cfg["F"], cfg["H"], rnn_type=cfg["rnn"])
    if cfg["plain"]:
        samp = M.Sampler(enc.hidden_size_total, cfg["Hm"], cfg["D"])
    else:
        samp = M.ABCDSampler(enc.hidden_size_total, cfg["Hm"], cfg["K"], cfg["D"])
    dec = M.RNN_Variational_Decoder(cfg["F"], cfg["H"], cfg["Hm"], cfg["D"], rnn_type=cfg["rnn"],
                                    num_speakers=cfg["spk"] or None, speaker_embed_dim=cfg["sdim"])
    for m in (enc, samp, dec):
        m.to(device).train()
    return engine.FusedStep(enc, samp, dec, device)


# The reference itself (ABCD-VAE/learning.py:147-163 on torch-CPU) cannot run on
# the GPU box; its measured throughput on the survey container (8 vCPU Xeon,
# 8 threads) is BASELINE.md's table, quoted beside the oracle-port timing.
REFERENCE_CPU = {
    "c2": {"value": 21.15, "range": [20.3, 22.0], "what": "ABCD LSTM b=512 T_max=200 F=129 K=128 h=256"},
    "c4": {"value": 24.0, "range": [24.0, 24.0], "what": "plain Gaussian-VAE LSTM, same shapes, f=16"},
    "c5": {"value": 4.2, "range": [4.2, 4.2], "what": "ABCD LSTM K=1024 T_max=512 (no speaker embedding)"},
    "c5gru": None,
}


# The same oracle sample timed in the survey container (8 vCPU Xeon, 8 torch
# threads) by scripts/cpu_calibrate.py: the box-to-box factor between the GPU
# box's host cores and the machine the reference's own CPU numbers
# (REFERENCE_CPU) were measured on ("CPU baseline calibration").
PORT_HERE = {  # round 4: python scripts/cpu_calibrate.py --threads 8 (b = 64 sample, same seeds as below)
    "c2": {"value": 31.221, "cores": 8}, "c4": {"value": 38.695, "cores": 8},
    "c5": {"value": 10.853, "cores": 8}, "c5gru": {"value": 12.172, "cores": 8},
}


def oracle_sample(cfg, b=64):
    """The bounded CPU sample of a workload: b segments of it, seed-1111
    weights, fixed replayed noise (oracle inputs)."""
    from oracle import abcd_oracle as O
    ocfg = O.default_cfg(F=cfg["F"], H=cfg["H"], Hdec=cfg["H"], Hm=cfg["Hm"], D=cfg["D"], K=cfg["K"] or 16,
                         rnn=cfg["rnn"], plain=cfg["plain"], fplain=cfg["D"],
                         num_speakers=cfg["spk"] or None, speaker_dim=cfg["sdim"])
    P = O.init_params(ocfg, 1111)
    sub = dict(cfg, B=b)
    batch = make_batch(sub, 4321, "cpu")
    g = torch.Generator().manual_seed(99)
    feat = torch.randn(b, cfg["D"], generator=g) if cfg["plain"] else \
        -torch.empty(b, cfg["K"]).exponential_(generator=g).log()
    eps = torch.randn(batch["L"], cfg["F"], generator=g)
    obatch = dict(data=batch["data"], batch_sizes=batch["batch_sizes"], is_offset=batch["is_offset"],
                  speakers=batch["speakers"])
    return dict(ocfg=ocfg, P=P, sub=sub, batch=batch, obatch=obatch, feat=feat, eps=eps, b=b)


def time_oracle(cfg, smp, target_s=10.0, budget_s=25.0, min_steps=3):
    """One untimed warm-up oracle step (returned: the parity anchor's
    reference), then timed steps until ~target_s of CPU work (at least
    min_steps, stopping past budget_s) -> (warm-up outputs, steps, seconds)."""
    from oracle import abcd_oracle as O
    noise = dict(feat=smp["feat"], eps=smp["eps"])
    ref, _, _, _, _ = O.train_step(smp["P"], smp["obatch"], smp["ocfg"], noise, cfg["N"])
    steps, t_total = 0, 0.0
    while steps < min_steps or (min_steps and t_total < target_s):
        t0 = time.perf_counter()
        O.train_step(smp["P"], smp["obatch"], smp["ocfg"], noise, cfg["N"])
        t_total += time.perf_counter() - t0
        steps += 1
        if t_total > budget_s:
            break
    return ref, steps, t_total


def cpu_baseline(cfg, cfg_name, device, target_s=10.0, budget_s=25.0, min_steps=3):
    """Time the CPU oracle on a bounded sample of the same workload: one
    untimed warm-up step, then b = 64 steps until ~target_s of CPU work
    (at least 3, stopping past budget_s).

    The warm-up step's outputs are also the parity anchor of the bench line:
    ONE HIP step on the same b = 64 sub-batch, weights (seed 1111 init order)
    and replayed noise gives the reconstruction-loss (Gaussian emission NLL,
    learning.py:153-157 ``em``) and total-loss relative deltas and the argmax
    category agreement.  Returns (cpu_baseline, parity)."""
    from modules import noise as _noise, engine as E
    threads = max(1, min(16, os.cpu_count() or 1))
    torch.set_num_threads(threads)
    smp = oracle_sample(cfg)
    b, sub, batch, feat, eps = smp["b"], smp["sub"], smp["batch"], smp["feat"], smp["eps"]
    bsz = batch["batch_sizes"]
    ref, steps, t_total = time_oracle(cfg, smp, target_s, budget_s, min_steps)
    rc = REFERENCE_CPU.get(cfg_name)
    value = round(steps * b / t_total, 3) if steps else None
    here = PORT_HERE.get(cfg_name)
    calib = None
    if here and value:
        ratio = value / here["value"]
        calib = {"port_here_seg_s": here["value"], "port_here_cores": here["cores"],
                 "box_over_here": round(ratio, 3),
                 "reference_on_box_est_seg_s": None if rc is None else round(rc["value"] * ratio, 2),
                 "what": "the same oracle sample timed in the container the reference's CPU numbers come from "
                         "(scripts/cpu_calibrate.py); reference_on_box_est = reference_cpu x box_over_here"}
    base = {"value": value, "calibration": calib, "unit": "segments/s", "cores": threads, "kind": "port",
            "sample": f"{steps} oracle train steps of b={b} segments (T_max={cfg['tmax']}, L={batch['L']} frames) "
                      f"of the {cfg['workload']} workload, torch-CPU fp32, {threads} threads",
            "reference_cpu_seg_s": None if rc is None else rc["value"],
            "reference_cpu": None if rc is None else dict(
                rc, unit="segments/s", cores=8, kind="reference",
                source="BASELINE.md: reference learning.py:147-163 timed in the survey container "
                       "(8 vCPU Xeon, 8 torch threads, b=512); the reference cannot run on the GPU box")}
    # --- parity anchor: one HIP step on the same sub-batch / weights / noise
    step = build(sub, device)
    _noise.replay(feat, eps)  # Gumbel (ABCD) or N(0,1) (plain) feature noise, then the decoder eps
    sc, logits = step.forward_backward(batch["data"].to(device), bsz, batch["is_offset"].to(device),
                                       batch["speakers"].to(device), cfg["N"])
    sc = sc.cpu()
    em_h, em_r = float(sc[E.EM]), float(ref["em"])
    lo_h, lo_r = float(sc[E.LOSS]), float(ref["loss"])
    parity = {"recon_loss_rel_delta": abs(em_h - em_r) / abs(em_r), "loss_rel_delta": abs(lo_h - lo_r) / abs(lo_r),
              "em_hip": em_h, "em_oracle": em_r, "sample": f"b={b} sub-batch of the workload (L={batch['L']}), "
              "seed-1111 weights, replayed noise; oracle = torch-CPU restatement pinned to the reference's "
              "fixtures (tests/golden)"}
    if not cfg["plain"]:
        lh, lr = logits.float().cpu(), ref["logits"].float()
        ah, ar = lh.argmax(-1), lr.argmax(-1)
        parity["argmax_equal"] = bool(torch.equal(ah, ar))
        parity["logits_max_abs_diff"] = float((lh - lr).abs().max())
        bad = (ah != ar).nonzero().flatten()
        parity["argmax_mismatch_rows"] = int(bad.numel())
        if bad.numel():  # the oracle's own gap between its top category and the HIP's pick: a near-tie?
            parity["argmax_tie_gap"] = float((lr[bad, ar[bad]] - lr[bad, ah[bad]]).max())
    del step
    return base, parity


def launch_ranks(n, argv):
    """``bench.py --gpus N`` with no WORLD_SIZE: run N ranks through
    torch.distributed.run as a child process (rendezvous on 127.0.0.1, one
    rank per GPU) and return its exit code.  Nothing here initialises the GPU
    (torch.cuda.device_count does not on this image), so the parent is never
    a GPU process that would have to be replaced."""
    import socket
    import subprocess
    if not os.environ.get("ABCD_BENCH_DRYRUN"):
        have = torch.cuda.device_count()
        if have < n:
            raise SystemExit(f"bench.py --gpus {n}: only {have} GPU(s) visible")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.call(cmd, env=env)


def dryrun_rank():
    """ABCD_BENCH_DRYRUN=1: a CPU stand-in for one bench rank (gloo, no GPU):
    checks the launcher's per-rank environment and prints what rank 0 sees.
    Used by the CPU test of the --gpus N launch path."""
    world = int(os.environ["WORLD_SIZE"])
    rank, local = int(os.environ["RANK"]), int(os.environ["LOCAL_RANK"])
    dist.init_process_group("gloo")
    t = torch.tensor([float(rank), float(local)])
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"dryrun": True, "world_size": dist.get_world_size(), "env_world": world,
                          "rank_sum": float(t[0]), "local_rank_sum": float(t[1]),
                          "master_addr": os.environ.get("MASTER_ADDR")}), flush=True)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (default: WORLD_SIZE under a launcher, else 1)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--batches", type=int, default=4, help="distinct synthetic batches cycled per rank")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    explicit = args.gpus is not None
    if not explicit:
        args.gpus = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if explicit and args.gpus != world:
        raise SystemExit(f"bench.py --gpus {args.gpus} under WORLD_SIZE={world}")
    if os.environ.get("ABCD_BENCH_DRYRUN"):
        return dryrun_rank()
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    from modules import noise, parallel, engine as E
    noise.set_mode("philox")
    noise.manual_seed(1234 + rank)
    step = build(cfg, device)
    if world > 1:
        parallel.broadcast_parameters(step)
        parallel.attach(step)
    batches = [make_batch(cfg, 1000 * rank + i, device) for i in range(args.batches)]
    lr, clip = 1.0, 1.0

    def run(i):
        b = batches[i % len(batches)]
        # weak scaling: the global batch is world x B segments; each rank
        # normalises by it and the gradient all-reduce sums (parallel.py)
        step.step(b["data"], b["batch_sizes"], b["is_offset"], b["speakers"], cfg["N"], is_pretraining=False,
                  lr=lr, momentum=0.0, clip=clip, loss_batch=world * cfg["B"])

    for i in range(args.warmup):
        run(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        run(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    # a persistent kernel that timed out invalidates the run (outside the timed region)
    from modules import _native as N
    N.raise_on_status(N.lib().abcd_device_status(), "bench")
    segs = world * cfg["B"] * args.steps
    value = segs / elapsed
    ms = elapsed / args.steps * 1e3
    Ls = [b["L"] for b in batches]
    L_avg = sum(Ls[i % len(Ls)] for i in range(args.steps)) / args.steps
    fl = flops_per_step(cfg, L_avg, cfg["B"])
    loss = float(step.scalars[E.LOSS])
    out = {
        "metric": "segments/sec/node (fwd+bwd), batch=512 K=128 h=256; recon-loss delta vs ref",
        "value": round(value, 2), "unit": "segments/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp32", "data": "synthetic (random STFT-shaped segments, random-init weights)",
        "config": {"workload": cfg["workload"], "global_batch": world * cfg["B"], "seq_len": cfg["tmax"],
                   "n_fft_bins": cfg["F"], "K": cfg["K"], "hidden": cfg["H"], "frames_per_batch_avg": L_avg,
                   "parallelism": f"dp{world}", "noise": "philox in-kernel", "final_loss": round(loss, 4)},
        "step_tflops": round(fl / (elapsed / args.steps) / 1e12, 3),
    }
    if world > 1:
        out["config"]["rccl_world_size"] = dist.get_world_size()
        out["allreduce_us_per_step"] = allreduce_time(step)
    if not args.no_kernel_timing:
        out["roofline"] = kernel_roofline(step, batches, cfg, run, args.config)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"], parity = cpu_baseline(cfg, args.config, device)
        out["recon_loss_rel_delta"] = parity["recon_loss_rel_delta"]
        out["parity"] = parity
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def allreduce_time(step, reps=10):
    """Mean time of the step's one collective (the SUM all-reduce of the flat
    fp32 gradient buffer, parallel.make_allreduce) on this rank, in us, max
    over ranks; bracketed by events on the current stream (the process
    group's collective is stream-ordered after it and waited for by it)."""
    g = step.flat.grad
    step.allreduce(g)
    torch.cuda.synchronize()
    dist.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        step.allreduce(g)
    e1.record()
    torch.cuda.synchronize()
    t = torch.tensor([e0.elapsed_time(e1) * 1e3 / reps], device=g.device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return round(float(t), 2)


def load_traffic(kernel, cfg_name):
    """HBM bytes per launch of `kernel` from the rocprofv3 PMC passes committed
    under profiles/ (scripts/pmc_traffic.py: FETCH_SIZE x 2 + WRITE_SIZE, the
    gfx950 correction of MI355X_MICROARCH.md) for this configuration, or None
    (no PMC pass of this configuration is committed).  One file per
    configuration: profiles/traffic_<config>.json (copied from the round's
    profiles/rNN/ set)."""
    path = os.path.join(REPO, "profiles", f"traffic_{cfg_name}.json")
    try:
        with open(path) as f:
            t = json.load(f)
        if t.get("config") != cfg_name:
            return None
        e = t["kernels"][kernel]
        return int(e["hbm_bytes_per_launch"])
    except (OSError, KeyError, ValueError):
        return None


def load_mfma(kernel, cfg_name):
    """MFMA utilisation of `kernel` from the rocprofv3 PMC pass committed under
    profiles/ (scripts/pmc_mfma.py: SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs x
    GRBM_GUI_ACTIVE / 8) for this configuration
    (profiles/pmc_mfma_<config>.json), or None."""
    path = os.path.join(REPO, "profiles", f"pmc_mfma_{cfg_name}.json")
    try:
        with open(path) as f:
            t = json.load(f)
        if t.get("config") != cfg_name:
            return None
        return float(t["kernels"][kernel]["mfma_busy"])
    except (OSError, KeyError, ValueError):
        return None


# The split-fp32 products (abcd_x6.h) issue 6 bf16 MFMAs per fp32 product:
# their instruction ceiling is the dense bf16 MFMA peak / 6 in fp32-equivalent FLOPs
PEAK_BF16_MFMA_TFLOPS = 16 * PEAK_FP32_MFMA_TFLOPS  # MI355X_MICROARCH.md: f32 MFMA = 1/16 of bf16
X6_CEILING_TFLOPS = PEAK_BF16_MFMA_TFLOPS / 6


def kernel_roofline(step, batches, cfg, run, cfg_name):
    """Roofline of the dominant kernel: the persistent recurrent kernel with
    the largest device time.  Its launches are bracketed live with HIP events
    on the launch stream by the library (abcd_timing_*); `achieved` =
    algorithmic FLOPs per launch (kernel_flops_per_frame x packed frames) /
    mean launch duration."""
    from modules import _native as N
    lib = N.lib()
    nsteps = 3
    lib.abcd_timing_reset()
    lib.abcd_timing_enable(1)
    for i in range(nsteps):
        run(i)
    torch.cuda.synchronize()
    lib.abcd_timing_enable(0)
    frames = [batches[i % len(batches)]["L"] for i in range(nsteps)]
    per = {}
    for kid, name in KERNELS.items():
        res = (N.c_double * 4)()
        lib.abcd_timing_read_kernel(kid, res)
        ms, launches = res[0], int(res[1])
        if launches == 0:
            continue
        fl = kernel_flops_per_frame(cfg, kid) * sum(frames) / launches
        avg_s = ms / 1e3 / launches
        per[name] = {"avg_launch_us": round(avg_s * 1e6, 3), "launches": launches,
                     "flops_per_launch": round(fl), "tflops": round(fl / avg_s / 1e12, 3)}
    if not per:
        return None
    dom = max(per, key=lambda k: per[k]["avg_launch_us"] * per[k]["launches"])
    d = per[dom]
    achieved = d["tflops"]
    traffic = load_traffic(dom, cfg_name)
    symbol = N.dispatch().get(dom, ("", 0))[0]
    return {"bound": "mfma", "kernel": dom, "kernel_symbol": "abcd::" + symbol if symbol else None,
            "achieved": achieved,
            "peak": PEAK_FP32_MFMA_TFLOPS,
            "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP32_MFMA_TFLOPS, 4), "traffic": traffic,
            "mfma_busy": load_mfma(dom, cfg_name),
            "x6_ceiling": {"peak": round(X6_CEILING_TFLOPS, 1), "frac": round(achieved / X6_CEILING_TFLOPS, 4),
                           "what": "bf16 dense MFMA peak / 6: the split-fp32 products' instruction ceiling"},
            "avg_launch_us": d["avg_launch_us"], "launches": d["launches"],
            "flops_per_launch": d["flops_per_launch"],
            # where each field comes from: achieved / frac are measured in THIS run;
            # traffic and mfma_busy are read from rocprofv3 PMC passes committed
            # under profiles/ (PMC counters cannot run inside the timed bench)
            "provenance": {"achieved": "live: HIP events on the launch stream, this run",
                           "traffic": f"committed profile: profiles/traffic_{cfg_name}.json"
                           if traffic is not None else None,
                           "mfma_busy": f"committed profile: profiles/pmc_mfma_{cfg_name}.json"
                           if load_mfma(dom, cfg_name) is not None else None},
            "all_kernels": per}


if __name__ == "__main__":
    main()
