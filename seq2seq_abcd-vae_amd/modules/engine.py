"""Fused training step: the body of ``Learner.train`` (ABCD-VAE/learning.py:147-163)
run as a fixed sequence of C-ABI calls, with no autograd graph.

    zero_grad -> encoder -> sampler.forward -> sample -> kl -> decoder
      -> loss = (em + off + kl) / batch_sizes[0] -> backward -> clip_grad_norm_ -> SGD

All parameters live in ONE flat fp32 device buffer (the modules' Parameters are
views into it, so ``state_dict``/checkpoints are unchanged) and all gradients
in a second one: the backward kernels write gradients in place, the global
clip + SGD is one pass over the flat buffers, and data parallelism is a single
all-reduce of the flat gradient buffer (``parallel.py``).  The step never
synchronises with the host; loss terms and diagnostics stay on the device in
``FusedStep.scalars`` until the caller reads them.
"""
import itertools

import torch

from . import _native as N
from . import noise as _noise
from . import padding as _pad
from .model import ABCDSampler

# layout of the device scalar vector returned by FusedStep.step; STATUS is the
# persistent kernels' timeout status of the step (abcd_step_status, non-zero =
# the step's results are invalid; check_status raises)
EM, OFF, KL, LOSS, NORM, PPL_CLUSTER, PPL_BATCH, PPL_SHAPE, STATUS = range(9)
N_SCALARS = 9
_SIDE_STREAMS = {}  # (device index, k) -> torch.cuda.Stream shared by every FusedStep (_side_stream)


class FlatParams:
    """Re-home a list of Parameters into one flat buffer (params) + one flat
    buffer (grads); each Parameter's ``.data``/``.grad`` become views."""

    def __init__(self, params, device):
        self.params = list(params)
        sizes = [p.numel() for p in self.params]
        self.offsets = list(itertools.accumulate([0] + sizes))[:-1]
        self.n = sum(sizes)
        self.flat = torch.empty(self.n, device=device)
        self.grad = torch.zeros(self.n, device=device)
        self.index = {}
        for p, o, s in zip(self.params, self.offsets, sizes):
            self.flat[o:o + s].copy_(p.detach().reshape(-1).to(device))
            p.data = self.flat[o:o + s].view_as(p)
            p.grad = self.grad[o:o + s].view_as(p)
            self.index[id(p)] = (o, s)

    def grad_of(self, p):
        o, s = self.index[id(p)]
        return self.grad[o:o + s].view_as(p)

    def rebind(self):
        """Re-attach .data/.grad views (e.g. after something replaced them)."""
        for p, o in zip(self.params, self.offsets):
            s = p.numel()
            if p.data.data_ptr() != self.flat[o:o + s].data_ptr():
                self.flat[o:o + s].copy_(p.data.reshape(-1))
                p.data = self.flat[o:o + s].view_as(p)
            if p.grad is None or p.grad.data_ptr() != self.grad[o:o + s].data_ptr():
                p.grad = self.grad[o:o + s].view_as(p)


class FusedStep:
    def __init__(self, encoder, sampler, decoder, device=None):
        self.encoder, self.sampler, self.decoder = encoder, sampler, decoder
        self.plain = not isinstance(sampler, ABCDSampler)
        device = torch.device(device) if device is not None else next(encoder.parameters()).device
        self.device = device
        params = itertools.chain(encoder.parameters(), sampler.parameters(), decoder.parameters())
        self.flat = FlatParams(params, device)
        # a size that is not a multiple of 16: the kernels run the zero-padded
        # twin model (padding.py); its parameters are embedded from self.flat
        # before every pass and its gradients gathered into self.flat.grad
        self.pad = None
        self.kmods = (encoder, sampler, decoder)  # the modules whose shapes the kernels run
        self.kflat = self.flat
        if _pad.PadPlan.needed(encoder, sampler, decoder):
            self.pad = _pad.PadPlan(encoder, sampler, decoder)
            self.kmods = self.pad.twins
            self.kflat = FlatParams(itertools.chain(*(m.parameters() for m in self.kmods)), device)
            self.kflat.flat.zero_()
            self.pad_index = self.pad.index.to(device)
            self.enc_cols = self.pad.dims[0].out_cols.to(device)
        self.momentum_buf = None
        self.momentum_init = True
        self._ws = {}
        self.optim_ws = N.workspace(N.lib().abcd_optim_workspace_bytes(self.flat.n), device)
        self.scalars = torch.zeros(N_SCALARS, device=device)
        self._inv = {}
        self._build_structs()
        self.allreduce = None  # set by parallel.DataParallel

    # ------------------------------------------------------------------ setup
    def _build_structs(self):
        (enc, samp, dec), fp = self.kmods, self.kflat
        self.enc_cfg = enc._cfg()
        self.enc_p = enc._params()
        dirs = 2 if enc.rnn.bidirectional else 1
        eg = {(l, d): [fp.grad_of(t) for t in enc.rnn.layer_weights(l, d)]
              for l in range(enc.rnn.num_layers) for d in range(dirs)}
        self.enc_g = enc._params(eg)
        self.samp_cfg = samp._scfg()
        self.samp_p = samp._sparams()
        views = {}
        for k, m in enumerate(samp._mlps()):
            for f, t in zip(("w1", "b1", "w2", "b2"), m.weights()):
                views[f"mlp{k}.{f}"] = fp.grad_of(t)
        if not self.plain:
            views["codebook"] = fp.grad_of(samp.codebook)
            views["posterior_shape_logits"] = fp.grad_of(samp.posterior_shape_logits)
        self.samp_g = samp._sgrads(views)
        self.dec_p = dec._dparams()
        self.dec_g = dec._dparams([fp.grad_of(t) for t in dec._param_list()])
        self.E = enc.hidden_size_total
        self.Dfeat = samp._feat_dim()

    def refresh(self):
        """Call after load_state_dict / .to(): re-bind views and pointer tables."""
        self.flat.rebind()
        if self.pad is not None:
            self.kflat.rebind()
        self._build_structs()

    def _workspace(self, name, nbytes):
        ws = self._ws.get(name)
        if ws is None or ws.numel() < nbytes:
            ws = N.workspace(int(nbytes * 1.1) + 4096, self.device)
            self._ws[name] = ws
        return ws

    def _inv_b(self, B):
        t = self._inv.get(B)
        if t is None:
            t = torch.full((), 1.0 / B, device=self.device)
            self._inv[B] = t
        return t

    # --------------------------------------------------------------- the step
    def forward_backward(self, data, batch_sizes, is_offset, speakers, entire_data_size, is_pretraining=False,
                         train=True, loss_batch=None):
        """Forward + backward of learning.py:149-158; gradients land in flat.grad.

        loss_batch: the loss normaliser (learning.py:156 ``batch_sizes[0]``).
        Default: this batch's B.  Under data parallelism every rank passes the
        GLOBAL batch size, so its loss is (em_r + off_r + kl_r) / B_global and
        the SUM of the ranks' gradients (and losses) is exactly the reference's
        global-batch value (parallel.py)."""
        if self.allreduce is not None and loss_batch is None:
            # a data-parallel rank normalising by its own B would scale the
            # summed gradient (and loss) by the world size
            raise ValueError("FusedStep with an all-reduce attached needs loss_batch = the GLOBAL batch size")
        L_ = N.lib()
        st = N.stream()
        data = data.contiguous()
        N.require_gpu(data)
        pk, bs_keep = _packed(data, batch_sizes, self.enc_cfg.input_size)
        T, L, B = pk.T, pk.L, pk.B
        Bn = int(loss_batch) if loss_batch is not None else B
        dev = self.device
        sc = self.scalars
        kenc, ksamp, kdec = self.kmods
        if self.pad is not None:  # this pass's weights into the padded twin (padding positions stay 0)
            self.kflat.flat.index_copy_(0, self.pad_index, self.flat.flat)
            for real, twin in zip((self.encoder, self.sampler, self.decoder), self.kmods):
                twin.train(real.training)
        ws_e = self._workspace("enc", L_.abcd_encoder_workspace_bytes(self.enc_cfg, T, L, B))
        ws_s = self._workspace("samp", L_.abcd_sampler_workspace_bytes(self.samp_cfg, B))
        dcfg = kdec._dcfg(None if train else 1)
        ws_d = self._workspace("dec", L_.abcd_decoder_workspace_bytes(dcfg, T, L, B))
        h = torch.empty(B, self.E, device=dev)
        # inter-layer dropout noise: the step's first RNG draw, as in the reference
        enc_noise = self.encoder.draw_dropout_noise(L, dev) if train else None
        if enc_noise is not None and self.pad is not None:
            de = self.pad.dims[0]
            enc_noise = [_pad.pad_col_blocks(n, de.dirs, de.H, de.Hp) for n in enc_noise]
        # the sampler's and the decoder's draws, in the reference's order, taken
        # up front (the decoder's Philox block is drawn inside its launch)
        W = ksamp._logit_width()
        if self.plain:
            mode, tau = 0, 1.0
            nt, seed, off = _noise.normal(B, self.sampler._feat_dim(), dev, width=self.Dfeat)
        elif is_pretraining:
            mode, tau, nt, seed, off = N.SAMPLE_SOFTMAX, 1.0, None, 0, 0
        else:
            mode, tau = N.SAMPLE_GUMBEL, float(self.sampler.temperature)
            nt, seed, off = _noise.gumbel(B, self.sampler._logit_width(), dev, width=W)
        F = kdec.rnn_cell.cell.input_size
        pdrop = self.decoder._input_dropout_p() if train else 0.0
        eps, eseed, eoff, xmask = _noise.decoder_noise(bs_keep, F, pdrop, dev)
        side = self._side_stream()
        side.wait_stream(torch.cuda.current_stream(dev))  # the previous step (parameters, eps) is queued before
        # the Dirichlet prior's per-category terms depend on the parameters
        # only: one small kernel on the side stream now, beside the input pack,
        # instead of in every sampler-head tile on the sampler's chain
        # (abcd_sampler_prior).  (Queued behind a noise fill it was dispatched
        # once the input projection held every CU -- that GEMM leaves no
        # registers for another workgroup -- and ran only as the projection
        # retired, beside the encoder's persistent launch.)
        prior = not self.plain
        if prior:
            N.check(L_.abcd_sampler_prior(self.samp_cfg, self.samp_p, B, float(entire_data_size), N.ptr(ws_s),
                                          ws_s.numel(), N.c_void_p(side.cuda_stream)), "sampler prior")
        # Philox mode (eps None): eps[row, f] = philox_normal(eseed, eoff + row * F + f),
        # drawn inside the decoder's persistent launch by its members without
        # an emit tile.  A side-stream fill here ran beside the input
        # projection (that GEMM holds every CU, so the fill was squeezed into
        # its tail, beside the encoder's persistent launch): same-box A/B at
        # c2, step 8.46 / 8.48 -> 8.39 / 8.43 ms, dec_fwd 2.24-2.25 -> 2.20 ms
        N.check(L_.abcd_encoder_forward_dropout(self.enc_cfg, self.enc_p, pk, N.ptr_array(enc_noise), N.ptr(h),
                                                N.ptr(ws_e), ws_e.numel(), st), "encoder forward")
        logits = torch.empty(B, W, device=dev)
        feats = torch.empty(B, self.Dfeat, device=dev)
        self._inspect(h, feats)  # kept for inspection (encode paths, parity tests)
        # feature_sampler(h) -> .sample(logits) -> .kl_divergence(logits, N)
        # (learning.py:149-153): ABCD = the split-K MLP GEMM + one row-tiled
        # sampler-head kernel (logits, Gumbel-softmax, y C^T, KL) per step
        if prior:
            torch.cuda.current_stream(dev).wait_stream(side)  # the prior stash (and the decoder noise)
        # (the cluster / batch perplexities stay in the head kernel's last
        # tile: a separate perplexity kernel on the side stream, placed before
        # dec_fwd or dec_bwd, held a CU one of their members then waited for --
        # 12-27 us of start skew -- for the ~5 us it saved here)
        N.check(L_.abcd_sampler_forward_fused(self.samp_cfg, self.samp_p, N.ptr(h), B,
                                              mode | (N.SAMPLE_PRIOR_READY if prior else 0), tau, N.ptr(nt), seed,
                                              off, float(entire_data_size), N.ptr(logits), N.ptr(feats),
                                              N.ptr(sc[KL:KL + 1]),
                                              None if self.plain else N.ptr(sc[PPL_CLUSTER:PPL_CLUSTER + 2]),
                                              N.ptr(ws_s), ws_s.numel(), st), "sampler")
        if not prior:  # (with the prior, the join in front of the sampler covered the noise:
            # a second, already-satisfied wait still cost a ~6 us barrier in front of the decoder)
            torch.cuda.current_stream(dev).wait_stream(side)  # the decoder noise
        spk = None
        if kdec.embed_speaker is not None:
            spk = speakers.to(dev, torch.int64).contiguous()
        gt_off = is_offset.contiguous()
        # the loss reductions (emission NLL, offset BCE, the total) only feed the
        # reported scalars: they run on the side stream beside the offset head
        side_p = N.c_void_p(side.cuda_stream)
        N.check(L_.abcd_decoder_forward_split(dcfg, self.dec_p, pk, N.ptr(feats), N.ptr(spk), N.ptr(gt_off),
                                              N.ptr(eps), N.ptr(xmask), eseed, eoff, None, None, None, None,
                                              N.ptr(sc[EM:EM + 2]), N.ptr(ws_d), ws_d.numel(), st, side_p),
                "decoder forward")
        N.check(L_.abcd_total_loss(N.ptr(sc[EM:EM + 2]), N.ptr(sc[KL:KL + 1]), Bn, N.ptr(sc[LOSS:LOSS + 1]),
                                   side_p), "total loss")
        if not train:
            torch.cuda.current_stream(dev).wait_stream(side)
            N.check(L_.abcd_step_status(N.ptr(sc[STATUS:STATUS + 1]), st), "step status")
            return sc, self._real_logits(logits)
        inv = self._inv_b(Bn)
        d_feats = torch.empty(B, self.Dfeat, device=dev)
        # the decoder's data-gradient path now; its weight-gradient reductions
        # (abcd_decoder_backward_params, below) are queued on the side stream
        # AFTER the encoder backward, to run beside it (joined before clip +
        # SGD: measured at c2 ~0.5 ms/step shorter than serial, DESIGN.md s3
        # Streams).  The gate armed here makes them wait, on the device, until
        # the encoder BPTT is resident on every CU; queuing them after that
        # launch means a side stream sharing its hardware queue cannot stall it.
        dargs = (dcfg, self.dec_p, pk, N.ptr(feats), N.ptr(spk), N.ptr(gt_off), N.ptr(xmask), N.ptr(inv), N.ptr(inv),
                 N.ptr(d_feats), self.dec_g, N.ptr(ws_d), ws_d.numel(), st)
        L_.abcd_side_gate_enable(1)
        try:
            N.check(L_.abcd_decoder_backward_dropout(*dargs, N.DEFER_PARAMS), "decoder backward")
        finally:
            L_.abcd_side_gate_enable(0)
        d_h = torch.empty(B, self.E, device=dev)
        # the sampler's codebook / W2 / W1 gradients (one batched launch) are
        # taken off the d_h -> enc_bwd chain (59-85 us there beside the
        # decoder's weight gradients) and queued after the encoder's backward
        # (31-38 us on a quiet chip; on the side stream behind the decoder's
        # weight gradients they ran beside gemm_wg3b and slowed it ~45 us)
        N.check(L_.abcd_sampler_backward_split(self.samp_cfg, self.samp_p, N.ptr(h), B, mode, tau,
                                               float(entire_data_size), N.ptr(d_feats), N.ptr(inv), N.ptr(d_h),
                                               self.samp_g, N.ptr(ws_s), ws_s.numel(), st, N.DEFER_PARAMS),
                "sampler backward")
        # (the encoder's own side work -- a GRU layer 0's backward-direction
        # weight gradients, forked after its BPTT -- on a second side stream,
        # so that the decoder's queued behind it below are not held back; the
        # LSTM's one-launch gemm_wg3b needs none, and an unused stream's join
        # would still cost a ~6 us barrier on the main stream)
        side2 = self._side_stream(1) if self.enc_cfg.rnn_type != N.LSTM else None
        N.check(L_.abcd_encoder_backward_dropout(self.enc_cfg, self.enc_p, pk, N.ptr_array(enc_noise), N.ptr(d_h),
                                                 self.enc_g, N.ptr(ws_e), ws_e.numel(), st,
                                                 N.c_void_p(side2.cuda_stream) if side2 is not None else None),
                "encoder backward")
        N.check(L_.abcd_decoder_backward_params(*dargs, side_p), "decoder weight gradients")
        N.check(L_.abcd_sampler_backward_params(self.samp_cfg, self.samp_p, N.ptr(h), B, self.samp_g, N.ptr(ws_s),
                                                ws_s.numel(), st, None), "sampler parameter gradients")
        torch.cuda.current_stream(dev).wait_stream(side)
        if side2 is not None:
            torch.cuda.current_stream(dev).wait_stream(side2)
        if self.pad is not None:  # the real positions of the twin's gradients
            torch.index_select(self.kflat.grad, 0, self.pad_index, out=self.flat.grad)
        return sc, self._real_logits(logits)

    def _real_logits(self, logits):
        """The real model's logits (ABCD: B x K; plain: [mean | log_var], B x 2f)
        from the kernels' (padded) ones."""
        if self.pad is None:
            return logits
        d = self.pad.dims[1]
        if not self.plain:
            return logits[:, :d.K]
        return torch.cat([logits[:, :d.D], logits[:, d.Dp:d.Dp + d.D]], 1)

    def _inspect(self, h, feats):
        """last_hidden / feats of the real model (views or gathers of the padded ones)."""
        if self.pad is None:
            self.last_hidden, self.feats = h, feats
            return
        self._padded_hidden, self._padded_feats = h, feats
        self.__dict__.pop("last_hidden", None)
        self.__dict__.pop("feats", None)

    def __getattr__(self, name):  # lazily gathered real views of the padded inspection tensors
        if name == "last_hidden" and "_padded_hidden" in self.__dict__:
            return self._padded_hidden.index_select(1, self.enc_cols)
        if name == "feats" and "_padded_feats" in self.__dict__:
            return self._padded_feats[:, :self.pad.dims[1].D]
        raise AttributeError(name)

    def _side_stream(self, k=0):
        """Side stream k (0: the step's side work, 1: the encoder backward's),
        one per device for the whole process: FusedSteps built one after the
        other reuse them instead of drawing new streams from torch's pool."""
        d = torch.device(self.device)
        key = (d.index if d.index is not None else torch.cuda.current_device(), k)
        s = _SIDE_STREAMS.get(key)
        if s is None:
            s = _SIDE_STREAMS[key] = torch.cuda.Stream(self.device)
        return s

    def optimizer_step(self, lr, momentum=0.0, clip=1.0):
        """clip_grad_norm_(all params, clip) + SGD(lr, momentum) on the flat buffers."""
        if self.allreduce is not None:
            self.allreduce(self.flat.grad)
        buf = None
        if momentum != 0.0:
            if self.momentum_buf is None:
                self.momentum_buf = torch.zeros_like(self.flat.flat)
                self.momentum_init = True
            buf = self.momentum_buf
        N.check(N.lib().abcd_clip_sgd(N.ptr(self.flat.flat), N.ptr(self.flat.grad), N.ptr(buf), self.flat.n,
                                      float(clip), float(lr), float(momentum), int(self.momentum_init),
                                      N.ptr(self.scalars[NORM:NORM + 1]), N.ptr(self.optim_ws),
                                      self.optim_ws.numel(), N.stream()), "clip+sgd")
        if buf is not None:
            self.momentum_init = False

    def empty_step(self, lr, momentum=0.0, clip=1.0):
        """A data-parallel rank whose shard of the global batch is empty: zero
        gradient and loss terms, but it still joins the all-reduce and applies
        the identical clip + SGD (so no rank waits on it)."""
        self.flat.grad.zero_()
        self.scalars.zero_()
        self.optimizer_step(lr, momentum, clip)
        return self.scalars

    def step(self, data, batch_sizes, is_offset, speakers, entire_data_size, is_pretraining=False, lr=1.0,
             momentum=0.0, clip=1.0, loss_batch=None):
        sc, logits = self.forward_backward(data, batch_sizes, is_offset, speakers, entire_data_size,
                                           is_pretraining, loss_batch=loss_batch)
        self.optimizer_step(lr, momentum, clip)
        if not self.plain:  # learning.py:171-178: cluster / batch perplexities came with the sampler head;
            # the shape perplexity reads posterior_shape_logits AFTER the SGD step
            N.check(N.lib().abcd_shape_perplexity(N.ptr(self.sampler.posterior_shape_logits), self.sampler.num_categories,
                                                  N.ptr(sc[PPL_SHAPE:PPL_SHAPE + 1]), N.stream()), "perplexities")
        N.check(N.lib().abcd_step_status(N.ptr(sc[STATUS:STATUS + 1]), N.stream()), "step status")
        return sc


def check_status(records, where="training step"):
    """Raise if any step's STATUS slot (rows of stacked scalar vectors, or
    one vector) is non-zero.  Call at a host read the caller already makes."""
    r = records.detach().reshape(-1, records.shape[-1])[:, STATUS]
    bad = r.nonzero()
    if bad.numel():
        N.raise_on_status(float(r[bad[0, 0]]), f"{where} {int(bad[0, 0]) + 1}")


class StatusWatch:
    """Bounded-latency check of the steps' STATUS slots inside an epoch.

    Every ``every`` steps the maximum STATUS of the records since the last
    check is reduced on the device and copied without blocking into pinned
    host memory; the copy of the PREVIOUS window is read (its event has long
    completed, so the host does not stall the stream) and a non-zero value
    raises ``PersistTimeout``.  A timed-out persistent kernel therefore stops
    training within two windows instead of at the end of the epoch, while
    the epoch loop still never synchronises with the device on the fast path.
    (The persistent kernels' own waits give up at once after a timeout, see
    ``spin_abandoned`` in abcd_persist.hip, so the steps in between are cheap.)
    """

    def __init__(self, device, every=16, where="training batch", group=None):
        """group: under data parallelism the process group whose ranks step
        together; each window's STATUS is MAX-reduced over it (one 4-byte
        all-reduce per window), so a timeout on one rank stops every rank."""
        self.every, self.where = int(every), where
        ws = torch.distributed.get_world_size(group) if torch.distributed.is_initialized() else 1
        self.group = group if ws > 1 else None
        if ws > 1 and group is None:
            self.group = torch.distributed.group.WORLD
        self.host = torch.zeros(1, pin_memory=torch.cuda.is_available())
        self.event = None
        self.first = 0   # first record of the window in flight
        self.done = 0    # records covered by the window in flight

    def _read(self):
        if self.event is not None:
            self.event.synchronize()
            if float(self.host[0]) != 0.0:
                N.raise_on_status(float(self.host[0]),
                                  f"{self.where}s {self.first + 1}-{self.done}")
            self.event = None

    def update(self, records):
        """records: the list of per-step scalar vectors of this epoch so far."""
        n = len(records)
        if n - self.done < self.every:
            return
        self._read()
        window = torch.stack(records[self.done:n])[:, STATUS].amax().reshape(1)
        if self.group is not None:  # every rank raises at the same batch (no rank left in the next all-reduce)
            torch.distributed.all_reduce(window, op=torch.distributed.ReduceOp.MAX, group=self.group)
        self.host.copy_(window, non_blocking=True)
        self.event = torch.cuda.Event()
        self.event.record()
        self.first, self.done = self.done, n

    def finish(self):
        self._read()


def _packed(data, batch_sizes, F):
    bs = batch_sizes
    if bs.dtype != torch.int64 or bs.device.type != "cpu":
        bs = bs.to("cpu", torch.int64)
    bs = bs.contiguous()
    st = N.Packed()
    st.data = data.data_ptr()
    st.batch_sizes = bs.data_ptr()
    st.T = int(bs.numel())
    st.L = int(data.shape[0])
    st.B = int(bs[0])
    st.F = int(F)
    return st, bs
