"""Native training loop: train_model() (VQ_VAE_HMM_fixed.py:145-162) and the
per-step executor it uses.

TrainState owns, per model:
  * one flat fp32 parameter buffer (the module's nn.Parameters become views of
    it, so state_dict()/checkpoints are unchanged) and a flat gradient buffer
    in vqhmm_param_layout order,
  * Adam moments + a device step counter (torch.optim.Adam defaults, :146),
  * a workspace per batch shape (B, T),
  * a device fp64 epoch accumulator: the loss is summed on the GPU in step
    order, so the epoch print needs ONE host sync per epoch instead of the
    reference's loss.item() every step (:158) — the printed value is the same
    double-precision sum of the same fp32 losses.

One step = elbo forward (+loss accumulate) -> elbo backward -> [RCCL
all-reduce of the flat gradient when torch.distributed is initialised] ->
fused Adam.  In a single process without clipping, Adam rides in the
backward's last launch (vqhmm_elbo_bwd_adam_f32).  Everything in the step is HIP kernels from libvqhmm.so plus the
collective; nothing syncs the host, so a fixed-shape step can be captured in a
HIP graph (`capture()`).  Optionally (overlap_bwd / VQHMM_BWD_OVERLAP=1) the
backward's weight gradients run on a side stream beside the data-gradient
chain (`_backward_overlapped`).
"""
import ctypes
import os
import sys

import torch

from . import _ext
from .model import _ptr_array, param_offsets

# Backward stage ids (csrc/api.hip `Stage`).  The data-gradient chain runs on the
# launch stream; each weight gradient runs on a side stream as soon as the chain
# stage that produces its dY has run (W_PAR only needs the forward's dpar).
S_PAR_DG, S_DEC2_DG, S_DEC1_DG, S_LOGIT_BWD, S_LOGIT_DG, S_ENC2_DG = 8, 9, 10, 11, 12, 13
S_W_PAR, S_W_DEC2, S_W_DEC1, S_W_LOGIT, S_W_ENC2, S_W_ENC1 = 14, 15, 16, 17, 18, 19
S_REDUCE, S_COMPOSE_BWD, S_LOGPRIOR = 20, 21, 22
BWD_CHAIN = ((S_PAR_DG, S_W_DEC2), (S_DEC2_DG, S_W_DEC1), (S_DEC1_DG, None), (S_LOGIT_BWD, S_W_LOGIT),
             (S_LOGIT_DG, S_W_ENC2), (S_ENC2_DG, S_W_ENC1))


def _overlap_default():
    # Off by default: measured on MI355X at cfg2 the overlapped step is slower
    # (0.702 vs 0.679 ms graphed, 0.686 vs 0.672 ms eager; profiles/r01/bwd_overlap_ab.txt):
    # every conv/wgrad kernel is persistent and already fills all 256 CUs, so
    # running two at once only adds contention.
    return os.environ.get("VQHMM_BWD_OVERLAP", "0") == "1"


class TrainState:
    def __init__(self, model, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, process_group=None, distributed=None,
                 overlap_bwd=None, dp_form=None):
        params = model.ordered_parameters()
        dev = params[0].device
        if dev.type != "cuda":
            raise RuntimeError("vqhmm.train_model runs on MI355X (HIP) only: call model.to('cuda') first")
        self.model = model
        self.device = dev
        self.dims = model._dims()
        self.off = param_offsets(self.dims)
        n = self.off[-1]
        self.flat = torch.empty(n, device=dev)
        with torch.no_grad():
            for i, p in enumerate(params):
                self.flat[self.off[i]:self.off[i + 1]].copy_(p.detach().reshape(-1))
                p.data = self.flat[self.off[i]:self.off[i + 1]].view_as(p)
        self.grad = torch.zeros(n, device=dev)
        self.exp_avg = torch.zeros(n, device=dev)
        self.exp_avg_sq = torch.zeros(n, device=dev)
        self.step_dev = torch.zeros((), dtype=torch.int64, device=dev)
        self.lr, self.betas, self.eps = float(lr), tuple(float(b) for b in betas), float(eps)
        self.ptrs = _ptr_array(params)
        self.loss = torch.zeros((), device=dev)
        self.epoch_acc = torch.zeros((), dtype=torch.float64, device=dev)
        self._ws = {}
        self._status = {}
        self.lib = _ext.load()
        if distributed is None:
            distributed = torch.distributed.is_available() and torch.distributed.is_initialized()
        self.distributed = bool(distributed)
        self.pg = process_group
        self.world = torch.distributed.get_world_size(process_group) if self.distributed else 1
        # the data-parallel step form (forward+backward, gradient all-reduce, Adam as its own launch):
        # needed with more than one rank; dp_form=True forces it on a 1-rank group (bench --dp-form)
        self.dp_form = (self.distributed and self.world > 1) if dp_form is None else bool(dp_form)
        if self.dp_form and not self.distributed:
            raise RuntimeError("vqhmm: dp_form needs an initialised torch.distributed process group")
        self.overlap_bwd = _overlap_default() if overlap_bwd is None else bool(overlap_bwd)
        self._side = None
        self._bwd_events = None

    # ----------------------------------------------------------------- helpers
    def workspace(self, B, T):
        key = (B, T)
        ws = self._ws.get(key)
        if ws is None:
            nb = ctypes.c_size_t()
            _ext.check(self.lib.vqhmm_elbo_workspace_size(ctypes.byref(self.dims), B, T, ctypes.byref(nb)),
                       "workspace")
            ws = torch.empty(nb.value, dtype=torch.uint8, device=self.device)
            off = ctypes.c_size_t()
            _ext.check(self.lib.vqhmm_elbo_status_offset(ctypes.byref(self.dims), B, T, ctypes.byref(off)),
                       "status offset")
            ws[off.value:off.value + 8].zero_()  # the kernels only ever set bits of it
            self._ws[key] = ws
            self._status[key] = ws[off.value:off.value + 8].view(torch.int64)
        return ws

    def check_status(self):
        """Raise if any step since the workspaces were made set a bit of the device status word
        (VQHMM_STATUS_*, e.g. the backward tail's bounded in-launch wait ran out).  Reads one
        8-byte word per workspace: call it where the host syncs anyway (once per epoch)."""
        for key, word in self._status.items():
            v = int(word.item())
            if v:
                what = "; ".join(m for b, m in _ext.STATUS_BITS.items() if v & b) or f"status 0x{v:x}"
                raise RuntimeError(f"vqhmm: training step (B, T) = {key} reported a device error: {what}")

    def prepare(self, x, u, lengths):
        dev = self.device
        x = x.to(dev, torch.float32, non_blocking=True).contiguous()
        u = u.to(dev, torch.float32, non_blocking=True).contiguous()
        lengths = torch.as_tensor(lengths).to(dev, torch.int64, non_blocking=True).contiguous()
        return x, u, lengths

    # -------------------------------------------------------------- the step
    def forward_backward(self, x, u, lengths, beta, norm=None):
        """Loss (accumulated into epoch_acc) and flat gradient of one batch.

        norm: None, or a device int64 {valid_count, batch} of the global batch this
        batch is a shard of (vqhmm.dist.global_norm); the loss and gradient are
        then this shard's share of the global batch's, and shares SUM to it."""
        B, _, T = x.shape
        lay = self.model.prior.u_layout(u)
        ws = self.workspace(B, T)
        st = _ext.stream_ptr(self.device)
        d = ctypes.byref(self.dims)
        # need_grad = 2: the loss is finalized in the backward's tail launch (vqhmm_elbo_bwd_loss_f32), one
        # launch fewer (the overlapped backward runs stage by stage, so its forward finalizes the loss itself)
        ng = 1 if self.overlap_bwd else 2
        _ext.check(self.lib.vqhmm_elbo_fwd_f32(d, self.ptrs, _ext.ptr(x), _ext.ptr(u), lay, _ext.ptr(lengths),
                                               _ext.ptr(norm), B, T, float(beta), ng, _ext.ptr(ws), ws.numel(),
                                               _ext.ptr(self.loss), _ext.ptr(self.epoch_acc), st), "elbo forward")
        if self.overlap_bwd:
            self._backward_overlapped(x, B, T, beta, ws, norm)
        else:
            _ext.check(self.lib.vqhmm_elbo_bwd_loss_f32(d, self.ptrs, _ext.ptr(x), _ext.ptr(norm), B, T, float(beta),
                                                        None, _ext.ptr(ws), ws.numel(), _ext.ptr(self.grad),
                                                        _ext.ptr(self.loss), _ext.ptr(self.epoch_acc), st),
                       "elbo backward")

    def _backward_overlapped(self, x, B, T, beta, ws, norm=None):
        """vqhmm_elbo_bwd_f32's stages with the weight gradients on a side stream.

        A wgrad only reads its chain dY buffer and saved activations and writes its
        own slabs, so each starts right after its dY is produced and runs beside the
        next dgrads; the side stream joins before reduce_slabs.  Same kernels, same
        fixed-order slab sums: bit-identical to the serial order.  Works eagerly and
        under HIP-graph capture (the fork/join become graph edges)."""
        main = torch.cuda.current_stream(self.device)
        if self._side is None:
            self._side = torch.cuda.Stream(self.device)
            self._bwd_events = [torch.cuda.Event() for _ in range(len(BWD_CHAIN) + 1)]
        side, ev = self._side, self._bwd_events
        d = ctypes.byref(self.dims)
        xp, wsp, gp, np_ = _ext.ptr(x), _ext.ptr(ws), _ext.ptr(self.grad), _ext.ptr(norm)

        def run(stage, stream):
            _ext.check(self.lib.vqhmm_elbo_stage_f32(d, self.ptrs, xp, None, 0, None, np_, B, T, float(beta), wsp,
                                                     ws.numel(), gp, stage, ctypes.c_void_p(stream.cuda_stream)),
                       "elbo backward")

        ev[0].record(main)
        side.wait_event(ev[0])
        run(S_W_PAR, side)
        k = 1
        for chain_stage, wgrad in BWD_CHAIN:
            run(chain_stage, main)
            if wgrad is not None:
                ev[k].record(main)
                side.wait_event(ev[k])
                run(wgrad, side)
                k += 1
        ev[k].record(side)
        main.wait_event(ev[k])
        for stage in (S_REDUCE, S_COMPOSE_BWD, S_LOGPRIOR):
            run(stage, main)

    def forward_backward_adam(self, x, u, lengths, beta, norm=None):
        """forward_backward + apply_adam with Adam fused into the backward's last launch
        (vqhmm_elbo_bwd_adam_f32): single process, no clipping."""
        B, _, T = x.shape
        lay = self.model.prior.u_layout(u)
        ws = self.workspace(B, T)
        st = _ext.stream_ptr(self.device)
        d = ctypes.byref(self.dims)
        # need_grad = 2: the loss is finalized in the backward's tail launch (one launch fewer)
        _ext.check(self.lib.vqhmm_elbo_fwd_f32(d, self.ptrs, _ext.ptr(x), _ext.ptr(u), lay, _ext.ptr(lengths),
                                               _ext.ptr(norm), B, T, float(beta), 2, _ext.ptr(ws), ws.numel(),
                                               _ext.ptr(self.loss), _ext.ptr(self.epoch_acc), st), "elbo forward")
        b1, b2 = self.betas
        rc = self.lib.vqhmm_elbo_bwd_adam_f32(d, self.ptrs, _ext.ptr(x), _ext.ptr(norm), B, T, float(beta),
                                              _ext.ptr(ws), ws.numel(), _ext.ptr(self.grad), _ext.ptr(self.flat),
                                              _ext.ptr(self.exp_avg), _ext.ptr(self.exp_avg_sq), self.lr, b1, b2,
                                              self.eps, _ext.ptr(self.step_dev), self.grad_scale(norm is not None),
                                              _ext.ptr(self.loss), _ext.ptr(self.epoch_acc), st)
        _ext.check(rc, "elbo backward + adam")

    def _fused_adam_ok(self, max_norm=None):
        return not self.dp_form and max_norm is None and not self.overlap_bwd

    def _step_device(self, x, u, lengths, beta, norm=None, max_norm=None):
        """One step on device tensors (no host sync)."""
        if self._fused_adam_ok(max_norm):
            self.forward_backward_adam(x, u, lengths, beta, norm)
            return
        self.forward_backward(x, u, lengths, beta, norm)
        self.reduce_gradients()
        if max_norm is None:
            self.apply_adam(global_norm=norm is not None)
        else:
            self.clip_grad_norm(max_norm, global_norm=norm is not None)
            self.apply_adam(scale=1.0)

    def reduce_gradients(self):
        if self.dp_form:
            torch.distributed.all_reduce(self.grad, op=torch.distributed.ReduceOp.SUM, group=self.pg)

    def grad_scale(self, global_norm=False):
        """Factor turning the (all-reduced) gradient buffer into the batch gradient: shards
        normalised by their own batch average over ranks (1/world); shards normalised by the
        global batch (global_norm) already sum to the global gradient (1)."""
        return 1.0 if global_norm else 1.0 / self.world

    def clip_grad_norm(self, max_norm, global_norm=False):
        """nn.utils.clip_grad_norm_(params, max_norm) on the flat gradient, on the device
        (src/training/trainer.py:32); leaves the gradient fully scaled (Adam then uses 1).
        The total norm (clip_grad_norm_'s return value) stays in self.total_norm."""
        if not hasattr(self, "total_norm"):
            self.total_norm = torch.zeros((), device=self.device)
        _ext.check(self.lib.vqhmm_clip_grad_norm_f32(_ext.ptr(self.grad), self.grad.numel(),
                                                     self.grad_scale(global_norm), float(max_norm),
                                                     _ext.ptr(self.total_norm), _ext.stream_ptr(self.device)),
                   "clip_grad_norm")
        return self.total_norm

    def apply_adam(self, global_norm=False, scale=None):
        """Adam on the (all-reduced) gradient, scaled by grad_scale() unless `scale` is given."""
        b1, b2 = self.betas
        scale = self.grad_scale(global_norm) if scale is None else float(scale)
        _ext.check(self.lib.vqhmm_adam_f32(_ext.ptr(self.flat), _ext.ptr(self.grad), _ext.ptr(self.exp_avg),
                                           _ext.ptr(self.exp_avg_sq), self.flat.numel(), self.lr, b1, b2, self.eps,
                                           _ext.ptr(self.step_dev), scale, _ext.stream_ptr(self.device)),
                   "adam")

    def step(self, x, u, lengths, beta, norm=None, max_norm=None):
        """zero_grad + compute_loss + backward + (all-reduce) + [clip_grad_norm_] + Adam.step
        (:154-157; with max_norm, Trainer.train_epoch's src/training/trainer.py:23-33).

        norm (device int64 {valid_count, batch} of the global batch, or None): see
        forward_backward.  With it, the ranks' summed gradient IS the global batch's."""
        x, u, lengths = self.prepare(x, u, lengths)
        self._step_device(x, u, lengths, beta, norm, max_norm)
        return self.loss

    def publish_grads(self):
        """Leave the last step's gradients in p.grad, as the reference loop does."""
        for i, p in enumerate(self.model.ordered_parameters()):
            p.grad = self.grad[self.off[i]:self.off[i + 1]].view_as(p).clone()

    def capture(self, x, u, lengths, beta, warmup=2, norm=None):
        """Capture one fixed-shape step into HIP graphs; returns a replay callable.

        Single process: the whole step is one graph.  Data-parallel form over RCCL:
        forward+backward, the gradient all-reduce and Adam captured as ONE graph; with
        gloo (which cannot be captured), a communicator that refuses capture, or
        VQHMM_DP_GRAPH=0: forward+backward and Adam are two graphs and the all-reduce
        runs between them from the host.  self.step_graphs says which (1 or 2)."""
        x, u, lengths = self.prepare(x, u, lengths)
        split = self.dp_form
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup):  # warm-up steps are real steps (identical to eager ones)
                self._step_device(x, u, lengths, beta, norm)
        torch.cuda.current_stream(self.device).wait_stream(s)
        if not split:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._step_device(x, u, lengths, beta, norm)
            self.step_graphs = 1
            return g.replay
        backend = str(torch.distributed.get_backend(self.pg))
        if backend == "nccl" and _dp_graph_default():
            # the whole DP step, RCCL all-reduce included, as ONE graph: no host hop between the
            # backward, the collective and Adam (B = 128 on one GPU, 1-rank RCCL group: 0.159 ->
            # 0.142 ms/step).  A communicator that refuses capture falls back to the split form.
            g = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(g):
                    self.forward_backward(x, u, lengths, beta, norm)
                    self.reduce_gradients()
                    self.apply_adam(norm is not None)
            except RuntimeError as e:  # pragma: no cover - depends on the RCCL build
                print(f"vqhmm: all-reduce could not be captured in the step graph ({e}); using split graphs",
                      file=sys.stderr)
            else:
                if self._verify_dp_graph(g, x, u, lengths, beta, norm):
                    self.step_graphs = 1
                    return g.replay
                print("vqhmm: the one-graph DP step differs from the eager step; using split graphs", file=sys.stderr)
        self.step_graphs = 2
        g_fb, g_adam = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_fb):
            self.forward_backward(x, u, lengths, beta, norm)
        with torch.cuda.graph(g_adam):
            self.apply_adam(norm is not None)

        def replay():
            g_fb.replay()
            self.reduce_gradients()
            g_adam.replay()
        return replay


    def _state_tensors(self):
        return [self.flat, self.grad, self.exp_avg, self.exp_avg_sq, self.step_dev, self.loss, self.epoch_acc]

    def _verify_dp_graph(self, g, x, u, lengths, beta, norm):
        """The one-graph DP step (RCCL all-reduce captured) checked once, on first use, against the eager
        DP step from the same state: parameters, moments, gradient and loss must agree bit for bit on every
        rank (one MAX all-reduce of the verdict, so all ranks pick the same form).  The state is restored
        afterwards, so the check costs two steps and changes nothing."""
        snap = [t.clone() for t in self._state_tensors()]
        g.replay()
        torch.cuda.synchronize(self.device)
        after_graph = [t.clone() for t in self._state_tensors()]
        for t, v in zip(self._state_tensors(), snap):
            t.copy_(v)
        self.forward_backward(x, u, lengths, beta, norm)
        self.reduce_gradients()
        self.apply_adam(norm is not None)
        torch.cuda.synchronize(self.device)
        same = all(torch.equal(a, b) for a, b in zip(after_graph, self._state_tensors()))
        for t, v in zip(self._state_tensors(), snap):
            t.copy_(v)
        bad = torch.tensor([0 if same else 1], dtype=torch.int32, device=self.device)
        torch.distributed.all_reduce(bad, op=torch.distributed.ReduceOp.MAX, group=self.pg)
        torch.cuda.synchronize(self.device)
        return int(bad.item()) == 0


def _dp_graph_default():
    # VQHMM_DP_GRAPH=0: the split form (fwd+bwd graph, all-reduce issued from the host, Adam graph), A/B
    return os.environ.get("VQHMM_DP_GRAPH", "1") != "0"


def train_model(model, dataloader, num_epochs=10, lr=1e-3):
    """Drop-in for VQ_VAE_HMM_fixed.train_model (:145-162): Adam(lr) with
    default betas/eps, beta warm-up min(1, 2(ep+1)/E), same epoch print."""
    state = TrainState(model, lr=lr)
    model.train()
    for ep in range(num_epochs):
        state.epoch_acc.zero_()
        beta = min(1.0, 2.0 * (ep + 1) / num_epochs)  # KL annealing
        for x, u, lengths in dataloader:
            state.step(x, u, lengths, beta)
        epoch_loss = state.epoch_acc.item()
        state.check_status()
        print(f"Epoch {ep+1}/{num_epochs}, Loss: {epoch_loss/len(dataloader):.4f}")
    state.publish_grads()
    return model


class Trainer:
    """Drop-in for the reference's Trainer (src/training/trainer.py:9-47): Adam(lr),
    compute_loss + backward + clip_grad_norm_(1.0) + step per batch, tqdm progress,
    `Epoch e/E, Loss: L, Beta: b` print.  Runs on TrainState (native HIP step, clip and
    Adam on the device); the epoch loss is accumulated on the device and read once
    per epoch (same double-precision sum of the same per-step losses as loss.item()).

    loss_fn(model, x, u, lengths) -> loss: a custom objective goes through autograd
    (vqhmm's compute_loss is differentiable); its parameter .grads are gathered into
    the flat gradient, then clipped and applied natively."""

    def __init__(self, model, lr=1e-3, device="cuda"):
        self.model = model.to(device)
        self.device = device
        self.state = TrainState(self.model, lr=lr)
        self.max_norm = 1.0

    def _custom_step(self, loss_fn, x, u, lengths):
        st = self.state
        x, u, lengths = st.prepare(x, u, lengths)
        params = self.model.ordered_parameters()
        for p in params:
            p.grad = None
        loss = loss_fn(self.model, x, u, lengths)
        loss.backward()
        with torch.no_grad():
            for i, p in enumerate(params):
                g = st.grad[st.off[i]:st.off[i + 1]]
                if p.grad is None:
                    g.zero_()
                else:
                    g.copy_(p.grad.reshape(-1))
            st.epoch_acc += loss.detach().double()
        st.reduce_gradients()
        st.clip_grad_norm(self.max_norm)
        st.apply_adam(scale=1.0)

    def train_epoch(self, dataloader, loss_fn=None, beta=1.0):
        try:
            from tqdm import tqdm
            it = tqdm(dataloader, desc="Training")
        except ImportError:  # progress bar only
            it = dataloader
        self.model.train()
        st = self.state
        st.epoch_acc.zero_()
        for x, u, lengths in it:
            if loss_fn is None:
                st.step(x, u, lengths, beta, max_norm=self.max_norm)
            else:
                self._custom_step(loss_fn, x, u, lengths)
        avg = st.epoch_acc.item() / len(dataloader)
        st.check_status()
        return avg

    def train(self, dataloader, num_epochs=100, use_beta_warmup=True):
        for ep in range(num_epochs):
            beta = min(1.0, 2.0 * (ep + 1) / num_epochs) if use_beta_warmup else 1.0
            avg_loss = self.train_epoch(dataloader, beta=beta)
            print(f"Epoch {ep+1}/{num_epochs}, Loss: {avg_loss:.4f}, Beta: {beta:.2f}")
        self.state.publish_grads()
