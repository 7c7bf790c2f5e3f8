"""Fused whole-model engine behind `VisionTransformer.forward` (the training hot path).

One autograd node covers the whole network: the forward (vit.py:77-80 -> transformer.py:76-79 per block ->
vit.py:69-74) runs as a fixed sequence of libvit_hip kernels on the current HIP stream and keeps every activation
the backward needs resident in HBM (ViT-B/16 at B=256 bf16: ~10 GB of 288 GB); the backward replays the block
sequence in reverse and writes every parameter gradient straight into ONE flat fp32 gradient buffer whose views are
exposed as `param.grad`.

Layouts (device):
  * master weights: the module's own fp32 nn.Parameters, untouched (state_dict/optimizer compatibility with the
    reference keys, including per-head `heads.{h}.{key,query,value}.weight`);
  * compute shadow: one buffer in the compute dtype holding, per block, the FUSED QKV matrix [3D, D] (query rows of
    every head, then keys, then values), proj [D, D], fc1 [4D, D], fc2 [D, 4D], and the patch-embedding matrix
    [D, C*P*P]; refreshed by the fused AdamW kernel (or a pack kernel after any external write);
  * gradients: one flat fp32 buffer ordered head | block L-1 | ... | block 0 | embedding, i.e. in the order the
    backward produces them, so data-parallel all-reduce buckets are contiguous ranges launched as soon as a block's
    backward is enqueued (RCCL on its own stream, overlapping the remaining backward).
"""
from __future__ import annotations

import math
import os
import weakref

import torch
import torch.distributed as dist
from torch.utils.weak import WeakIdKeyDictionary

from . import _lib, _ops
from ._ops import ACT_NONE, ACT_RELU

# parameter -> its compute-dtype shadow view (refreshed by FusedAdamW's kernel).  Kept beside the parameters, not as
# attributes on them, so models stay picklable / deep-copyable (torch.save(model), EMA snapshots).
SHADOWS = WeakIdKeyDictionary()


def shadow_of(p):
    return SHADOWS.get(p)


DROPOUT_P = 0.2          # transformer.py:35,53 (config.dropout is stored but unused by the reference)
LN_EPS = 1e-5
ALIGN = 64               # elements; every sub-tensor of the flat buffers starts 256-B aligned


def _hash_u32(seed, idx):
    """Python twin of the device `vit_hash_u32` (murmur3 fmix32 of idx*golden + seed)."""
    x = (idx * 0x9E3779B1 + seed) & 0xFFFFFFFF
    x ^= x >> 16
    x = (x * 0x85EBCA6B) & 0xFFFFFFFF
    x ^= x >> 13
    x = (x * 0xC2B2AE35) & 0xFFFFFFFF
    x ^= x >> 16
    return x


def site_seed(base_seed, layer, site):
    """Dropout seed of (layer, site); site 0 = MHA output (transformer.py:47), 1 = FFN output (:59)."""
    return _hash_u32((base_seed * 0x632BE5AB + 0x1234567) & 0xFFFFFFFF, layer * 2 + site)


def dropout_seed(base_seed, rank=0):
    """Base dropout seed of one forward on data-parallel replica `rank`: the seed drawn from the CPU RNG, with the
    rank hashed in for rank > 0 (rank 0 keeps the single-process seed, so a one-rank job is bitwise a plain run).
    Each replica's masks are then a different counter-hash stream, as independent torch bernoulli draws per rank
    would be (transformer.py:40,59 under an 8-way split of the batch)."""
    if rank == 0:
        return base_seed
    return _hash_u32((base_seed ^ 0x5BD1E995) & 0xFFFFFFFF, 0x27D4EB2F + rank) & 0x7FFFFFFF


class _Region:
    def __init__(self):
        self.size = 0
        self.items = []

    def add(self, name, numel):
        off = self.size
        self.items.append((name, off, numel))
        self.size = off + ((numel + ALIGN - 1) // ALIGN) * ALIGN
        return off


def split_k_for(m, n, k, dtype=torch.bfloat16):
    """K split for a weight-gradient GEMM (reduction over B*T rows), chosen by the library for the kernel it will
    run (vit_gemm_split_k_hint: one round of output tiles x K-slices over the 256 CUs)."""
    return int(_lib.load().vit_gemm_split_k_hint(m, n, k, _ops.dtype_code(dtype)))


def head_split_for(m, n, k):
    """K split for the classifier head's fp32 GEMMs (M = batch rows only): ~1024 workgroups of the 64x64 fp32
    tile, each slice >= 4 k-steps of 32 (128 k).  Without it these few-tile GEMMs run one long dependent k-loop per
    CU."""
    tiles = ((m + 63) // 64) * ((n + 63) // 64)
    nkt = (k + 31) // 32
    return max(1, min((1024 + tiles - 1) // tiles, nkt // 4, 32))


class Tape:
    """Activations saved by a training forward."""
    __slots__ = ("B", "cols", "blocks", "z", "u", "gz", "zn", "mh", "rh", "seed", "training", "x_shape", "x_dtype",
                 "x_grad", "pruned", "row0")


class Engine:
    def __init__(self, model):
        self.model_ref = weakref.ref(model)
        cfg = model.vit_config
        self.C, self.P = cfg.input_channels, cfg.patch_size
        self.D, self.H, self.L = cfg.embedding_size, cfg.num_heads, cfg.num_blocks
        self.hd = self.D // self.H
        self.N = cfg.num_patches
        self.T = self.N + 1
        self.nc = cfg.num_classes
        self.B = cfg.batch_size
        self.CPP = self.C * self.P * self.P
        self.dtype = model.compute_dtype
        self.scale = float(self.hd) ** 0.5          # MULTIPLIED (transformer.py:24)
        self.device = None
        self.params = None
        self.ddp_group = None
        self.ddp_enabled = False
        # dtype the gradient buckets travel in over RCCL (enable_data_parallel(grad_dtype=...)): fp32, or bf16 (half
        # the ring bytes; the buffer is averaged in bf16 and widened back into the fp32 gradients)
        self.comm_dtype = torch.float32
        # when set (bench.py, last timed step): HIP events around the bucket waits at the end of the backward, i.e.
        # the communication time the backward did not hide ("exposed"); read with comm_exposed_ms()
        self.time_comm = False
        self._comm_events = None
        self._works = []
        self._ws = None
        self._tok = None
        self._ptr_sig = None
        self._ver_sig = None
        self.stats = {"packs": 0}
        # callable(family, phase, flop, nbytes) around the hot launches (bench.py's live HIP-event roofline):
        # phase 0 before the launch with its algorithmic FLOPs / HBM bytes, phase 1 after it, same stream
        self.profile_hook = None
        # roctx ranges named by kernel family around the same launches (torch.cuda.nvtx is roctx on ROCm): visible in
        # `rocprofv3 --marker-trace` timelines.  Off by default (a host call per launch).
        self.trace_ranges = False
        # weight-gradient GEMMs on a side stream (an attribute for A/B runs and tests).  On by default since round 5:
        # interleaved A/B on one box, ViT-B/16 B=256: 31.53 vs 32.05 ms/step (profiles/r9g_concurrent_wgrad_ab.log;
        # in round 1, with slower kernels, it had measured 41.3 vs 40.5 ms and was left off)
        self.concurrent_wgrad = True
        # the forward's encoder blocks as two half-batch chains on two HIP streams (_forward_blocks_split): each fills
        # the other's idle CUs (partial last rounds of tiles, kernel drains); outputs bitwise those of one chain
        self.fwd_streams = 2
        self._split_fwd = False
        self._fwd_pair = None
        # backward kernels share the CUs with RCCL collectives (set by enable_data_parallel on the nccl backend;
        # an attribute, so A/B runs can force either launch mode)
        self.shared_cus = False
        self._wstream = None
        self._wws = None
        # the last block's post-attention part on the B token-0 rows only (see forward); False: every row (tests)
        self.prune_last = True
        # ... and its attention on query 0 alone (vit_attn_fwd_row0 / vit_attn_bwd_row0); False: the full attention
        # kernels with the output gradient zero outside row 0 (A/B runs; set it between steps, not between a forward
        # and its backward)
        self.row0_attention = True
        # data-parallel replica index folded into the dropout seed (enable_data_parallel sets the group rank): every
        # rank draws the same base seed from its identically seeded CPU RNG, so without it all replicas would apply
        # the same keep masks to different images.  0 (rank 0, single process) leaves the seed unchanged.
        self.dropout_rank = 0
        # .grad views set at the end of backward() instead of its start when every grad was None (_attach_grads);
        # an attribute for A/B runs
        self.defer_grad_attach = True
        self._pending_views = None

    # ------------------------------------------------------------------------------------------------------------
    # layout
    # ------------------------------------------------------------------------------------------------------------
    def _collect(self, model):
        """name -> Parameter for the fused layout, following the reference module tree."""
        enc = model.transformer_encoder.blocks
        emb = model.emdeddings
        p = {"conv_w": emb.sequence[0].weight, "conv_b": emb.sequence[0].bias,
             "cls": emb.cls_tkn_embd, "pos": emb.pos_embd,
             "h0_w": model.mlp[0].weight, "h0_b": model.mlp[0].bias,
             "hln_w": model.mlp[2].weight, "hln_b": model.mlp[2].bias,
             "h3_w": model.mlp[3].weight, "h3_b": model.mlp[3].bias}
        for l, blk in enumerate(enc):
            mh = blk.multi_head
            for h, head in enumerate(mh.heads):
                p[f"{l}.q{h}"] = head.query.weight
                p[f"{l}.k{h}"] = head.key.weight
                p[f"{l}.v{h}"] = head.value.weight
            p[f"{l}.proj_w"], p[f"{l}.proj_b"] = mh.proj.weight, mh.proj.bias
            p[f"{l}.fc1_w"], p[f"{l}.fc1_b"] = blk.ffwd.mlp[0].weight, blk.ffwd.mlp[0].bias
            p[f"{l}.fc2_w"], p[f"{l}.fc2_b"] = blk.ffwd.mlp[2].weight, blk.ffwd.mlp[2].bias
            p[f"{l}.ln1_w"], p[f"{l}.ln1_b"] = blk.ln1.weight, blk.ln1.bias
            p[f"{l}.ln2_w"], p[f"{l}.ln2_b"] = blk.ln2.weight, blk.ln2.bias
        return p

    def _build(self, model, device):
        D, H, hd, L = self.D, self.H, self.hd, self.L
        params = self._collect(model)
        for n, t in params.items():
            if t.dtype != torch.float32 or not t.is_contiguous():
                raise RuntimeError(f"parameter {n} must be contiguous float32 master weights (got {t.dtype})")
            if t.device != device:
                raise RuntimeError(f"parameter {n} is on {t.device}, expected {device}; call model.to(device)")
        # ---- gradient layout: head | blocks L-1..0 | embedding
        g = _Region()
        goff = {}
        head_start = g.size
        for n in ("h0_w", "h0_b", "hln_w", "hln_b", "h3_w", "h3_b"):
            goff[n] = g.add(n, params[n].numel())
        self.head_range = (head_start, g.size)
        self.block_range = {}
        for l in reversed(range(L)):
            start = g.size
            goff[f"{l}.qkv_w"] = g.add(f"{l}.qkv_w", 3 * D * D)
            for n in ("proj_w", "proj_b", "fc1_w", "fc1_b", "fc2_w", "fc2_b", "ln1_w", "ln1_b", "ln2_w", "ln2_b"):
                goff[f"{l}.{n}"] = g.add(f"{l}.{n}", params[f"{l}.{n}"].numel())
            self.block_range[l] = (start, g.size)
        start = g.size
        for n in ("conv_w", "conv_b", "cls", "pos"):
            goff[n] = g.add(n, params[n].numel())
        self.embed_range = (start, g.size)
        self.G = torch.zeros(g.size, dtype=torch.float32, device=device)
        # ---- compute shadow layout
        s = _Region()
        soff = {}
        for l in range(L):
            soff[f"{l}.qkv_w"] = s.add(f"{l}.qkv_w", 3 * D * D)
            for n in ("proj_w", "fc1_w", "fc2_w"):
                soff[f"{l}.{n}"] = s.add(f"{l}.{n}", params[f"{l}.{n}"].numel())
        soff["conv_w"] = s.add("conv_w", params["conv_w"].numel())
        self.W = torch.empty(s.size, dtype=self.dtype, device=device)

        def gview(name, shape):
            o = goff[name]
            n = math.prod(shape)
            return self.G[o:o + n].view(shape)

        def wview(name, shape):
            o = soff[name]
            n = math.prod(shape)
            return self.W[o:o + n].view(shape)

        # fused compute/grad views
        self.gw, self.ww = {}, {}
        for l in range(L):
            self.gw[f"{l}.qkv_w"] = gview(f"{l}.qkv_w", (3 * D, D))
            self.ww[f"{l}.qkv_w"] = wview(f"{l}.qkv_w", (3 * D, D))
            for n in ("proj_w", "fc1_w", "fc2_w"):
                shp = tuple(params[f"{l}.{n}"].shape)
                self.gw[f"{l}.{n}"] = gview(f"{l}.{n}", shp)
                self.ww[f"{l}.{n}"] = wview(f"{l}.{n}", shp)
            for n in ("proj_b", "fc1_b", "fc2_b", "ln1_w", "ln1_b", "ln2_w", "ln2_b"):
                self.gw[f"{l}.{n}"] = gview(f"{l}.{n}", tuple(params[f"{l}.{n}"].shape))
        for n in ("h0_w", "h0_b", "hln_w", "hln_b", "h3_w", "h3_b", "conv_b", "cls", "pos"):
            self.gw[n] = gview(n, tuple(params[n].shape))
        self.gw["conv_w"] = gview("conv_w", (D, self.CPP))
        self.ww["conv_w"] = wview("conv_w", (D, self.CPP))

        # per-parameter grad view + shadow view (the optimizer refreshes the shadow in its kernel)
        self.grad_views = []
        self.grad_region = []           # gradient region (key of self.gw / self.owners) of each grad view
        self.pack_entries = []
        for name, p in params.items():
            l, _, short = name.partition(".") if "." in name else ("", "", name)
            if short and short[0] in "qkv" and short[1:].isdigit():
                h = int(short[1:])
                row0 = {"q": 0, "k": D, "v": 2 * D}[short[0]] + h * hd
                gv = self.gw[f"{l}.qkv_w"][row0:row0 + hd]
                sv = self.ww[f"{l}.qkv_w"][row0:row0 + hd]
                self.grad_region.append(f"{l}.qkv_w")
            else:
                key = name
                gv = self.gw[key].view(p.shape)
                sv = self.ww[key].view(p.shape) if key in self.ww else None
                self.grad_region.append(key)
            self.grad_views.append((p, gv))
            SHADOWS[p] = sv
            if sv is not None:
                self.pack_entries.append((p, sv))
        self.params = params
        self.param_list = list(params.values())
        # which parameters feed each gradient region (a fused QKV region serves 3H per-head parameters)
        self.owners = {}
        for name, p in params.items():
            l, _, short = name.partition(".") if "." in name else ("", "", name)
            key = f"{l}.qkv_w" if (short and short[0] in "qkv" and short[1:].isdigit()) else name
            self.owners.setdefault(key, []).append(p)
        self.device = device
        self._pack_table = None
        self._ptr_sig = self._pointer_signature()
        self._ver_sig = None

    def _pointer_signature(self):
        return tuple(p.data_ptr() for p in self.param_list)

    def _version_signature(self):
        return sum(p._version for p in self.param_list)

    def ensure_ready(self, device):
        model = self.model_ref()
        if model is None or getattr(model, "_engine", None) is not self:
            raise RuntimeError("this engine does not belong to the model it is called for (copied engine?); "
                               "models must build their own engine (VisionTransformer.hip_engine)")
        if self.params is None or self.device != device or self._pointer_signature() != self._ptr_sig:
            self._build(model, device)
        ver = self._version_signature()
        if ver != self._ver_sig:
            self.repack()
            self._ver_sig = ver

    def repack(self):
        """shadow <- compute-dtype copy of the fp32 master matrices (one multi-tensor launch)."""
        if self._pack_table is None:
            entries = [(p.detach(), None, None, None, sv) for p, sv in self.pack_entries]
            self._pack_table = _ops.build_chunk_table(entries, self.device)
        tab, n = self._pack_table
        _ops.pack(tab, n, self.dtype)
        self.stats["packs"] += 1

    def mark_shadow_fresh(self):
        self._ver_sig = self._version_signature()

    # ------------------------------------------------------------------------------------------------------------
    def _token_rows(self, name, M, D, dt, T, dev):
        """[M, D] buffer that is zero outside the token-0 rows b*T (the pruned last block's attention-backward operands):
        allocated zeroed once per shape; every use writes exactly rows b*T again, so the rest stays zero and no
        M x D fill runs per step."""
        key = (name, M, D, dt, T, dev)
        buf = self._tok.get(key) if self._tok is not None else None
        if buf is None:
            if self._tok is None:
                self._tok = {}
            buf = self._tok[key] = torch.zeros(M, D, dtype=dt, device=dev)
        return buf

    def _workspace(self, nbytes):
        if self._ws is None or self._ws.numel() * 4 < nbytes:
            self._ws = torch.empty(max(nbytes // 4 + 1, 1 << 20), dtype=torch.float32, device=self.device)
        return self._ws

    def _side_stream(self):
        """HIP stream for the weight-gradient GEMMs of the backward (None: run them in order on the current stream).
        A weight gradient depends only on tensors the current stream has already produced and nothing reads it
        before the bucket all-reduce / the optimizer step, so on its own stream it runs beside the dgrad / attention
        / LayerNorm chain and fills the CUs that chain leaves idle (partial last rounds of tiles, memory-bound
        kernels).  Same kernels, same inputs: the gradients are bitwise those of the in-order schedule."""
        if not self.concurrent_wgrad or self.device is None or self.device.type != "cuda":
            return None
        if self._wstream is None or self._wstream.device != self.device:
            self._wstream = torch.cuda.Stream(device=self.device)
        return self._wstream

    def _mark(self, fam, phase, flop=0.0, nbytes=0.0):
        h = self.profile_hook
        if h is not None:
            h(fam, phase, flop, nbytes)
        if self.trace_ranges:
            if phase == 0:
                torch.cuda.nvtx.range_push(fam)
            else:
                torch.cuda.nvtx.range_pop()

    def _wgrad(self, dy, x, out, m, n, k, ld_dy, ld_x, beta, side=None, fam=None, alpha=1.0):
        """out[m][n] (+)= alpha sum_r dy[r][i] x[r][j]: weight gradient, reduction over B*T rows, split-K.  With `side`
        it runs on that stream after everything already enqueued on the current one."""
        split = split_k_for(m, n, k, dy.dtype)
        need = split * m * n * 4 if split > 1 else 0
        if side is None:
            ws = self._workspace(need) if split > 1 else None
            if fam:
                self._mark(fam, 0, 2.0 * m * n * k, (m + n) * k * dy.element_size() + m * n * 4 * (1 + (beta != 0)))
            _ops.gemm(dy, x, out, m, n, k, ld_dy, ld_x, out.stride(0), a_kcontig=False, b_kcontig=False, beta=beta,
                      alpha=alpha, split_k=split, workspace=ws)
            if fam:
                self._mark(fam, 1)
            return
        side.wait_stream(torch.cuda.current_stream(self.device))
        ws = None
        if need:
            if self._wws is None or self._wws.numel() * 4 < need:
                self._wws = torch.empty(max(need // 4 + 1, 1 << 20), dtype=torch.float32, device=self.device)
            ws = self._wws
        _ops.gemm(dy, x, out, m, n, k, ld_dy, ld_x, out.stride(0), a_kcontig=False, b_kcontig=False, beta=beta,
                  alpha=alpha, split_k=split, workspace=ws, stream=side)
        for t in (dy, x) if ws is None else (dy, x, ws):
            t.record_stream(side)          # the caching allocator must not hand these out before `side` is done

    def _gemm_rows(self, pr, a, b, c, m, n, k, lda, ldb, ldc, **kw):
        """A token-row GEMM; `pr` (the pruned last block, m = B rows): split-K over the otherwise idle CUs — a few
        256x256 tiles would each run one long k-loop on one CU.  (Two-stream forward: each call gets its own slabs,
        allocated on its stream, instead of the shared workspace.)"""
        split = split_k_for(m, n, k, a.dtype) if pr else 1
        if split > 1:
            kw.update(split_k=split, workspace=None if self._split_fwd else self._workspace(split * m * n * 4))
        return _ops.gemm(a, b, c, m, n, k, lda, ldb, ldc, **kw)

    @staticmethod
    def _rows_of(bufs, b0, B, T):
        """rows(name, token0): this call's slice (images b0 .. b0+B-1) of the whole-batch buffer bufs[name] — T rows
        per image, or one (token0: the pruned block's token-0 rows); lse by image.  None without bufs."""
        def rows(name, token0=False):
            if bufs is None:
                return None
            t = bufs[name]
            per = 1 if (token0 or name == "lse") else T
            return t[b0 * per:(b0 + B) * per]
        return rows

    @staticmethod
    def _mask4_out(bufs, name, r0, R, n, dev):
        """A VIT_MASK4 buffer for rows r0 .. r0+R-1 of an [.., n] tensor: fresh, or that byte range of bufs[name]
        (4-row groups: r0 and R multiples of 4)."""
        if bufs is None:
            return _ops.mask4_empty(R, n, dev)
        off = (r0 // 4) * ((n + 3) // 4) * 4
        return bufs[name][off:off + _ops.mask4_bytes(R, n)]

    def _gemm_bwd(self, *args, **kw):
        """A backward GEMM that may overlap the bucket all-reduce (launch mode: self.shared_cus)."""
        return _ops.gemm(*args, shared_cus=self.shared_cus, **kw)

    def _head_gemm(self, a, b, c, m, n, k, lda, ldb, ldc, **kw):
        split = head_split_for(m, n, k)
        ws = self._workspace(split * m * n * 4) if split > 1 else None
        _ops.gemm(a, b, c, m, n, k, lda, ldb, ldc, split_k=split, workspace=ws, **kw)

    def _head_linear(self, x, w, bias):
        m, k = x.shape
        n = w.shape[0]
        y = torch.empty(m, n, dtype=x.dtype, device=x.device)
        self._head_gemm(x, w, y, m, n, k, x.stride(0), w.stride(0), n, bias=bias)
        return y

    def _colsum(self, x, rows, cols, ld, out, beta, alpha=1.0):
        _ops.colsum(x, rows, cols, ld, out, beta=beta, alpha=alpha)

    def _attach_grads(self):
        """Expose the flat gradient buffer as param.grad of every parameter that requires grad (frozen ones keep
        .grad untouched, as autograd would); returns beta (1.0 accumulate / 0.0 overwrite)."""
        views = [(p, gv) for p, gv in self.grad_views if p.requires_grad]
        live = [p.grad is not None and p.grad.data_ptr() == gv.data_ptr() for p, gv in views]
        if all(live):
            return 1.0
        if not any(p.grad is not None for p, _ in views):
            if not self.defer_grad_attach:
                for p, gv in views:
                    p.grad = gv
                return 0.0
            # the common case after zero_grad(set_to_none=True): the ~0.3 ms of .grad setter calls is deferred to
            # the end of backward() (_attach_pending), after the head and block kernels are enqueued — host work off
            # the forward -> backward turn, where a profiled run (slower launches) left the GPU idle; nothing reads
            # the views before then (interleaved A/B without a profiler: within noise, profiles/r22_*)
            self._pending_views = views
            return 0.0
        # mixed: zero the regions whose grad was dropped/replaced, keep accumulating elsewhere
        for (p, gv), ok in zip(views, live):
            if not ok:
                if p.grad is not None:
                    gv.copy_(p.grad)
                else:
                    gv.zero_()
                p.grad = gv
        return 1.0

    def _attach_pending(self):
        views, self._pending_views = self._pending_views, None
        for p, gv in views or ():
            p.grad = gv

    # ------------------------------------------------------------------------------------------------------------
    # forward
    # ------------------------------------------------------------------------------------------------------------
    def forward(self, x, training, save, want_probs=False):
        if not x.is_cuda:
            raise RuntimeError("VisionTransformer (HIP path) needs the input on a ROCm device; there is no CPU path")
        if x.dim() != 4 or x.shape[1] != self.C or x.shape[2] % self.P or x.shape[3] % self.P:
            raise RuntimeError(f"expected input [B, {self.C}, H, W] with H, W multiples of {self.P}, got "
                               f"{tuple(x.shape)}")
        B = x.shape[0]
        self.ensure_ready(x.device)
        if (x.shape[2] // self.P) * (x.shape[3] // self.P) != self.N:
            raise RuntimeError(f"image gives {(x.shape[2] // self.P) * (x.shape[3] // self.P)} patches but "
                               f"config.num_patches = {self.N} (pos_embd has {self.T} rows)")
        if B != self.params["cls"].shape[0]:
            # the reference concatenates a batch-shaped CLS parameter (vit.py:32,41) and fails the same way
            raise RuntimeError(f"batch size {B} != config.batch_size {self.params['cls'].shape[0]} "
                               "(the CLS token parameter is batch-shaped)")
        x = x.contiguous()
        if x.dtype not in (torch.float32, torch.bfloat16):
            x = x.float()
        D, T, N, L, dt = self.D, self.T, self.N, self.L, self.dtype
        M = B * T
        es = 2 if dt == torch.bfloat16 else 4
        prm = self.params
        mk = self._mark
        seed = dropout_seed(int(torch.randint(0, 2 ** 31 - 1, (1,)).item()), self.dropout_rank) if training else 0
        tape = Tape() if save else None

        blocks = []
        # The classifier reads token 0 of the last block's output only (vit.py:80), and everything after the last
        # attention is per token: the last block's proj / LN2 / MLP (and their backward) run on the B token-0 rows
        # (rows b*T, row stride T*D; dropout bits drawn at the full tensor's indices) — the same logits, loss and
        # gradients as computing all B*T rows and discarding the rest.  `prune_last = False` computes every row.
        prune = self.prune_last
        nc = self.fwd_streams
        cols = torch.empty(B * N, self.CPP, dtype=dt, device=x.device)
        xcur = torch.empty(M, D, dtype=dt, device=x.device)
        if (nc > 1 and not want_probs and self.profile_hook is None and B % (4 * nc) == 0
                and ((B // nc) * T) % 4 == 0):
            xcur = self._forward_blocks_split(x, cols, xcur, B, training, seed, save, prune, blocks, nc)
        else:
            self._embed(x, cols, xcur, 0, B)
            for l in range(L):
                xcur, saved = self.block_forward(l, xcur, B, training, seed, save, want_probs, prune and l == L - 1)
                if save:
                    blocks.append(saved)
        # classifier on token 0 (= first PATCH, vit.py:80): Linear -> GELU(erf) -> LayerNorm(4D) -> Linear, fp32
        z = torch.empty(B, D, dtype=torch.float32, device=x.device)
        _ops.copy2d(xcur, D if prune else T * D, z, D, B, D)
        u = self._head_linear(z, prm["h0_w"], prm["h0_b"])
        gz = _ops.gelu_fwd(u)
        zn, mh, rh = _ops.layernorm_fwd(gz, prm["hln_w"], prm["hln_b"], eps=LN_EPS)
        logits = self._head_linear(zn, prm["h3_w"], prm["h3_b"])
        if save:
            tape.B, tape.cols, tape.blocks = B, cols, blocks
            tape.x_shape, tape.x_dtype = tuple(x.shape), x.dtype
            tape.z, tape.u, tape.gz, tape.zn, tape.mh, tape.rh = z, u, gz, zn, mh, rh
            tape.seed, tape.training, tape.pruned = seed, training, prune
            # which attention the pruned block's forward ran (query 0 alone, or the full kernels): its backward must
            # be the matching one whatever row0_attention says by then (the row-0 forward writes only rows b*T)
            tape.row0 = prune and self.row0_attention and not want_probs
        return logits, tape

    def _block_bufs(self, B, training, save, dev):
        """Whole-batch outputs of one (unpruned) block for the two-stream forward: the tensors block_forward would
        allocate."""
        D, T, H, hd, dt = self.D, self.T, self.H, self.hd, self.dtype
        M = B * T
        e = lambda *shape, dtype=dt: torch.empty(*shape, dtype=dtype, device=dev)   # noqa: E731
        f32 = torch.float32
        b = {"a1": e(M, D), "m1": e(M, dtype=f32), "r1": e(M, dtype=f32), "qkv": e(M, 3 * D), "o": e(M, D),
             "lse": e(B, H, T, dtype=f32), "x_mid": e(M, D), "a2": e(M, D), "m2": e(M, dtype=f32),
             "r2": e(M, dtype=f32), "h": e(M, 4 * D), "x_out": e(M, D)}
        if save and _ops.attn_bwd_uses_o32(B, T, H, hd, dt):
            b["o32"] = e(M, D, dtype=f32)
        if save and training:
            b["pm"] = _ops.mask4_empty(M, D, dev)
            b["fm"] = _ops.mask4_empty(M, D, dev)
        if save:
            b["hm"] = _ops.mask4_empty(M, 4 * D, dev)
        return b

    def _embed(self, x, cols, xcur, b0, B):
        """Patch embedding (vit.py:21-29, 39-42) of images b0 .. b0+B-1 into their rows of the whole-batch cols /
        xcur: im2col, the conv as a GEMM with conv bias + pos and the (b, n) -> b*T + n row remap in its epilogue,
        then the CLS rows (appended LAST, vit.py:41)."""
        D, T, N, dt = self.D, self.T, self.N, self.dtype
        es = 2 if dt == torch.bfloat16 else 4
        prm = self.params
        cl = cols[b0 * N:(b0 + B) * N]
        xc = xcur[b0 * T:(b0 + B) * T]
        _ops.im2col(x[b0:b0 + B], self.P, dt, cols=cl)                                # vit.py:21-29 as GEMM
        self._mark("gemm_fwd", 0, 2.0 * B * N * D * self.CPP, (B * N + D) * self.CPP * es + B * N * D * es)
        _ops.gemm(cl, self.ww["conv_w"], xc, B * N, D, self.CPP, self.CPP, self.CPP, D, bias=prm["conv_b"],
                  res=prm["pos"].view(T, D), ldres=D, res_rowmod=N, out_group=(N, T))  # + pos, rows -> b*T+n
        self._mark("gemm_fwd", 1)
        _ops.embed_cls(prm["cls"].reshape(-1, D)[b0:b0 + B], prm["pos"], xc, B, T, D)  # CLS appended LAST

    def _forward_blocks_split(self, x, cols, xcur, B, training, seed, save, prune, blocks, nc=2):
        """The patch embedding and the encoder blocks as nc chains of B/nc images on nc HIP streams (default two),
        into the whole-batch cols / xcur allocated on the current stream, up to the last block's output, which the
        current stream then waits for.  Every kernel is the one-chain forward's on a row range (rows are
        independent; dropout indices are the whole batch's), so the outputs are bitwise the same; the chains fill
        each other's idle CUs.  The blocks' outputs are whole-batch buffers allocated on the current stream and
        recorded on every chain stream."""
        D, T, L = self.D, self.T, self.L
        dev = xcur.device
        cur = torch.cuda.current_stream(dev)
        if self._fwd_pair is None or len(self._fwd_pair) != nc or self._fwd_pair[0].device != dev:
            self._fwd_pair = tuple(torch.cuda.Stream(device=dev) for _ in range(nc))
        streams = self._fwd_pair
        for st in streams:
            st.wait_stream(cur)
        Bh, Mh = B // nc, (B // nc) * T
        for t in (x, cols, xcur):
            for st in streams:
                t.record_stream(st)
        for i, st in enumerate(streams):
            with torch.cuda.stream(st):
                self._embed(x, cols, xcur, i * Bh, Bh)
        names = ("a1", "m1", "r1", "qkv", "o", "o32", "lse", "x_mid", "a2", "m2", "r2", "h", "hm", "pm", "fm")
        # the ring attention forward of one chain on 3/4 of the CUs, so the other chain's GEMMs run beside it instead
        # of waiting for the whole latency-bound kernel (one box, interleaved: 30.50 -> 30.19 ms/step; 1/2 and 7/8 of
        # the CUs gain less) — unless the caller set the attn_fwd_grid option itself.  Passed per call (vit_attn_fwd's
        # max_wgs, ABI 14): no process-wide state changes, so concurrent forwards on other threads are unaffected.
        wgs = 0
        if _lib.get_option("attn_fwd_grid") == 0:
            wgs = max(1, torch.cuda.get_device_properties(dev).multi_processor_count * 3 // 4)
        self._split_fwd = True
        # the pruned last block runs whole-batch after the join: split, its B token-0 rows would become two GEMMs of
        # B/2 rows (below the 256-row tile: the slow small-M kernels)
        nsplit = L - 1 if prune else L
        # without a tape (no_grad / eval) nothing outlives the next block: two buffer sets, ping-ponged.  Each chain
        # reads and writes only its own rows, in order on its own stream, so block l + 2 may overwrite block l's rows
        # of a chain once that chain's block l + 1 consumed them (fresh sets per block, each recorded on
        # both streams, let the caching allocator hold up to L blocks of activations while the host runs ahead)
        ping = None if save else [self._block_bufs(B, training, save, dev) for _ in range(2)]
        for t in ([xcur] if save else [xcur] + [t for bs in ping for t in bs.values()]):
            for st in streams:
                t.record_stream(st)
        try:
            for l in range(nsplit):
                if save:
                    bufs = self._block_bufs(B, training, save, dev)
                    for t in bufs.values():
                        for st in streams:
                            t.record_stream(st)
                else:
                    bufs = ping[l % 2]
                for i, st in enumerate(streams):
                    with torch.cuda.stream(st):
                        self.block_forward(l, xcur[i * Mh:(i + 1) * Mh], Bh, training, seed, save, False, False,
                                           bufs=bufs, b0=i * Bh, attn_wgs=wgs)
                if save:
                    blocks.append((xcur,) + tuple(bufs.get(n) for n in names))
                xcur = bufs["x_out"]
        finally:
            self._split_fwd = False
        pre = None
        if nsplit < L and self.row0_attention:
            # the pruned block's ln1 and K / V GEMM are whole-row work: per chain too
            l = L - 1
            D = self.D
            pre = (torch.empty(B * T, D, dtype=self.dtype, device=dev),
                   torch.empty(B * T, dtype=torch.float32, device=dev),
                   torch.empty(B * T, dtype=torch.float32, device=dev),
                   torch.empty(B * T, 3 * D, dtype=self.dtype, device=dev))
            for t in pre:
                for st in streams:
                    t.record_stream(st)
            wq = self.ww[f"{l}.qkv_w"]
            for i, st in enumerate(streams):
                r = slice(i * Mh, (i + 1) * Mh)
                with torch.cuda.stream(st):
                    _ops.layernorm_fwd(xcur[r], self.params[f"{l}.ln1_w"], self.params[f"{l}.ln1_b"], eps=LN_EPS,
                                       y=pre[0][r], mean=pre[1][r], rstd=pre[2][r])
                    _ops.gemm(pre[0][r], wq[D:], pre[3][r][:, D:], Mh, 2 * D, D, D, D, 3 * D)
        for st in streams:
            cur.wait_stream(st)
        if nsplit < L:
            xcur, saved = self.block_forward(L - 1, xcur, B, training, seed, save, False, True, pre=pre)
            if save:
                blocks.append(saved)
        return xcur

    def block_forward(self, l, x_in, B, training, seed, save, want_probs=False, pr=False, bufs=None, b0=0,
                      pre=None, attn_wgs=0):
        """Block l (transformer.py:76-79) on x_in [B*T, D] (compute dtype): x_mid = x_in + drop(MHA(ln1(x_in))),
        x_out = x_mid + drop(FFN(ln2(x_mid))).  `pr`: the post-attention part on the B token-0 rows only (the pruned
        last block).  Returns (x_out, saved): `saved` is what block_backward needs (None unless `save`).
        `bufs` (the two-stream forward, _forward_blocks_split): the block's outputs for the whole batch, preallocated;
        this call is images b0 .. b0+B-1 of it and writes their rows (dropout bits drawn at the whole batch's
        indices), saved = None.  `pre` (the pruned block after the two-chain forward): its ln1 output / statistics and
        qkv with the K / V columns already computed per chain; only the token-0 rows' Q GEMM is left."""
        model = self.model_ref()
        D, T, H, hd, dt = self.D, self.T, self.H, self.hd, self.dtype
        M = B * T
        es = 2 if dt == torch.bfloat16 else 4
        prm = self.params
        mk = self._mark
        drop_p = DROPOUT_P if training else 0.0
        keep_masks = save and training          # the backward reads the forward's dropout keep bits (mask4)
        dev = x_in.device
        blk = model.transformer_encoder.blocks[l]
        ln_b = 2 * M * D * es + 8 * M
        mk("ln_fwd", 0, 0.0, ln_b)
        rows = self._rows_of(bufs, b0, B, T)                  # this call's slice of a whole-batch buffer
        q0only = pr and self.row0_attention and not want_probs  # the pruned block's attention on query 0 alone
        wq = self.ww[f"{l}.qkv_w"]
        if pre is not None:
            a1, m1, r1, qkv = pre
            mk("ln_fwd", 1)
        else:
            a1, m1, r1 = _ops.layernorm_fwd(x_in, prm[f"{l}.ln1_w"], prm[f"{l}.ln1_b"], eps=LN_EPS,
                                            y=rows("a1"), mean=rows("m1"), rstd=rows("r1"))
            mk("ln_fwd", 1)
        if q0only:
            # ... which reads Q of the token-0 rows only: K / V of every row (one GEMM into columns D..3D), Q of the
            # B token-0 rows (split-K over the idle CUs); the other Q rows of qkv are never read
            if pre is None:
                qkv = rows("qkv") if bufs is not None else torch.empty(M, 3 * D, dtype=dt, device=dev)
                mk("gemm_fwd", 0, 2.0 * M * 2 * D * D, (M * D + 2 * D * D + 2 * M * D) * es)
                _ops.gemm(a1, wq[D:], qkv[:, D:], M, 2 * D, D, D, D, 3 * D)
                mk("gemm_fwd", 1)
            mk("gemm_fwd", 0, 2.0 * B * D * D, (2 * B * D + D * D) * es)
            self._gemm_rows(True, a1, wq, qkv, B, D, D, T * D, D, T * 3 * D)
            mk("gemm_fwd", 1)
        else:
            mk("gemm_fwd", 0, 2.0 * M * 3 * D * D, (M * D + 3 * D * D + 3 * M * D) * es)
            qkv = _ops.linear(a1, wq) if bufs is None else _ops.gemm(a1, wq, rows("qkv"), M, 3 * D, D, D, D, 3 * D)
            mk("gemm_fwd", 1)
        probs = None
        if want_probs:
            probs = torch.empty(B, H, T, T, dtype=torch.float32, device=dev)
        if q0only:
            # the pruned last block: only attention output row 0 of every image is read (the classifier reads token 0,
            # everything after the attention is per token), and every softmax row is independent -> query 0 alone,
            # O(T hd) per (image, head); o rows b*T and lse[:, :, 0] are written
            o32 = None
            mk("attn_fwd", 0, 4.0 * B * H * T * hd, 2 * M * D * es + 2 * B * D * es + 4 * B * H)
            o, lse = _ops.attn_fwd_row0(qkv, B, T, H, hd, self.scale, o=rows("o"), lse=rows("lse"))
            mk("attn_fwd", 1)
        else:
            # training forward in bf16 with the tiled (T > 256) backward: also keep O unrounded for its exact delta;
            # the fused T <= 256 backward forms delta from P and dP itself (vit_hip.h)
            o32 = None
            if save and _ops.attn_bwd_uses_o32(B, T, H, hd, dt):
                o32 = rows("o32") if bufs is not None else torch.empty(M, D, dtype=torch.float32, device=dev)
            mk("attn_fwd", 0, 4.0 * B * H * T * T * hd, 4 * M * D * es + 4 * B * H * T + (4 * M * D if o32 is not None
                                                                                         else 0))
            o, lse = _ops.attn_fwd(qkv, B, T, H, hd, self.scale, o=rows("o"), lse=rows("lse"), probs=probs, o32=o32,
                                   max_wgs=attn_wgs)
            mk("attn_fwd", 1)
        blk.multi_head.attention_probs = probs
        blk.multi_head._probs_skipped = probs is None       # a later read warns once (transformer.py)
        # rows of the post-attention part: all M, or (last block, pruned) the B token-0 rows b*T
        R, rs = (B, T) if pr else (M, 1)
        r0 = b0 if pr else b0 * T                                     # this call's first row of the whole batch
        pm = self._mask4_out(bufs, "pm", r0, R, D, dev) if keep_masks else None      # proj dropout keep bits
        fm = self._mask4_out(bufs, "fm", r0, R, D, dev) if keep_masks else None      # fc2 dropout keep bits
        x_mid = rows("x_mid", pr) if bufs is not None else torch.empty(R, D, dtype=dt, device=dev)
        mk("gemm_fwd", 0, 2.0 * R * D * D, (3 * R * D + D * D) * es)
        self._gemm_rows(pr, o, self.ww[f"{l}.proj_w"], x_mid, R, D, D, rs * D, D, D, bias=prm[f"{l}.proj_b"],
                        res=x_in, ldres=rs * D, dropout_p=drop_p, seed=site_seed(seed, l, 0),
                        drop_row_stride=rs, mask_out=pm, drop_row0=r0)
        mk("gemm_fwd", 1)
        mk("ln_fwd", 0, 0.0, 2 * R * D * es + 8 * R)
        a2, m2, r2 = _ops.layernorm_fwd(x_mid, prm[f"{l}.ln2_w"], prm[f"{l}.ln2_b"], eps=LN_EPS,
                                        y=rows("a2", pr), mean=rows("m2", pr), rstd=rows("r2", pr))
        mk("ln_fwd", 1)
        # saved for the backward: the ReLU mask as 1 bit per element (mask4, read by fc2's dgrad epilogue instead
        # of re-reading h: 1/16 of the bytes)
        hm = self._mask4_out(bufs, "hm", r0, R, 4 * D, dev) if save else None
        mk("gemm_fwd", 0, 2.0 * R * 4 * D * D, (R * D + 4 * D * D + 4 * R * D) * es + (R * D // 2 if save else 0))
        h = rows("h", pr) if bufs is not None else torch.empty(R, 4 * D, dtype=dt, device=dev)
        self._gemm_rows(pr, a2, self.ww[f"{l}.fc1_w"], h, R, 4 * D, D, D, D, 4 * D, bias=prm[f"{l}.fc1_b"],
                        act=ACT_RELU, mask_out=hm)
        mk("gemm_fwd", 1)
        x_out = rows("x_out", pr) if bufs is not None else torch.empty(R, D, dtype=dt, device=dev)
        mk("gemm_fwd", 0, 2.0 * R * 4 * D * D, (4 * R * D + 4 * D * D + 2 * R * D) * es)
        self._gemm_rows(pr, h, self.ww[f"{l}.fc2_w"], x_out, R, D, 4 * D, 4 * D, 4 * D, D, bias=prm[f"{l}.fc2_b"],
                        res=x_mid, ldres=D, dropout_p=drop_p, seed=site_seed(seed, l, 1), drop_row_stride=rs,
                        mask_out=fm, drop_row0=r0)
        mk("gemm_fwd", 1)
        saved = (x_in, a1, m1, r1, qkv, o, o32, lse, x_mid, a2, m2, r2, h, hm, pm, fm) if save and bufs is None \
            else None
        return x_out, saved

    # ------------------------------------------------------------------------------------------------------------
    # backward
    # ------------------------------------------------------------------------------------------------------------
    def _bucket_ready(self, rng, side=None):
        """Launch the all-reduce of one contiguous gradient range (RCCL stream waits on the compute stream, and on
        the weight-gradient stream `side` when there is one).  With comm_dtype bf16 the range is first rounded into
        a bf16 buffer (on the stream that produced it), which is what travels and is averaged."""
        if not self.ddp_enabled:
            return
        a, b = rng
        bf = self.comm_dtype == torch.bfloat16
        nccl = dist.get_backend(self.ddp_group) == "nccl"
        if nccl:                                          # RCCL: native average
            if side is not None:                          # issued from `side`: the main chain does not wait
                side.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(side):
                    buf = self.G[a:b].to(torch.bfloat16) if bf else self.G[a:b]
                    w = dist.all_reduce(buf, op=dist.ReduceOp.AVG, group=self.ddp_group, async_op=True)
            else:
                buf = self.G[a:b].to(torch.bfloat16) if bf else self.G[a:b]
                w = dist.all_reduce(buf, op=dist.ReduceOp.AVG, group=self.ddp_group, async_op=True)
            self._works.append((w, rng, buf if bf else None, False))
        else:                                             # gloo (CPU tests): sum, scaled after the wait
            if side is not None:
                torch.cuda.current_stream(self.device).wait_stream(side)
            buf = self.G[a:b].to(torch.bfloat16) if bf else self.G[a:b]
            w = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.ddp_group, async_op=True)
            self._works.append((w, rng, buf if bf else None, True))

    def _finish_buckets(self):
        if not self._works:
            return
        world = dist.get_world_size(self.ddp_group) if self.ddp_enabled else 1
        ev = None
        if self.time_comm and self.device is not None and self.device.type == "cuda":
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()                      # every backward kernel is enqueued before this point
        for w, (a, b), buf, scale in self._works:
            w.wait()                            # nccl: the current stream waits for the collective
            if buf is not None:
                self.G[a:b].copy_(buf)          # bf16 average -> fp32 gradients
                if buf.is_cuda:                 # may have been allocated on the weight-gradient stream
                    buf.record_stream(torch.cuda.current_stream(buf.device))
            if scale:
                self.G[a:b].mul_(1.0 / world)
        if ev is not None:
            ev[1].record()
        self._comm_events = ev
        self._works = []

    def comm_exposed_ms(self):
        """Milliseconds the compute stream spent, after the last backward kernel, waiting for the gradient
        all-reduce of the most recent backward with time_comm set (None if not measured).  Synchronizes."""
        if self._comm_events is None:
            return None
        self._comm_events[1].synchronize()
        return self._comm_events[0].elapsed_time(self._comm_events[1])

    def backward(self, tape, dlogits):
        D, T, N, L, dt = self.D, self.T, self.N, self.L, self.dtype
        B = tape.B
        M = B * T
        prm, gw = self.params, self.gw
        # decided at backward time: the reference calls zero_grad(set_to_none=True) between forward and backward
        self._pending_views = None
        beta = self._attach_grads()
        # Accumulating into existing .grad (no zero_grad between backwards) with `register_hook` hooks present:
        # autograd applies such a hook to THIS backward's gradient only, then accumulates.  Keep the old gradients
        # aside, let the kernels overwrite the buffer with the increment (beta 0), and let run_param_hooks() hook
        # the increment and add the old values back (old + increment is the same single fp32 rounding the beta=1
        # epilogues do, so hook-free parameters keep their bits).
        self._acc_old = None
        if beta == 1.0 and any(p.requires_grad and p._backward_hooks for p, _ in self.grad_views):
            self._acc_old = self.G.clone()
            beta = 0.0
        req = {k: any(p.requires_grad for p in ps) for k, ps in self.owners.items()}
        # a frozen per-head parameter whose .grad is still a view of G shares the fused QKV gradient region with the
        # heads that do train; that region is rewritten as a whole, so keep the frozen view's value aside (autograd
        # leaves a frozen parameter's .grad untouched).  Only such views: a region whose owners are all frozen is
        # never written.
        self._frozen_keep = [] if self._acc_old is not None else [
            (gv, gv.clone()) for (p, gv), key in zip(self.grad_views, self.grad_region)
            if not p.requires_grad and req[key] and p.grad is not None and p.grad.data_ptr() == gv.data_ptr()]
        # the backward stops at the first block below which nothing (parameters, input image) needs a gradient
        below = tape.x_grad or any(req[k] for k in ("conv_w", "conv_b", "cls", "pos"))
        need_from = {}
        for l in range(L):
            below = below or any(req[f"{l}.{n}"] for n in ("qkv_w", "proj_w", "proj_b", "fc1_w", "fc1_b", "fc2_w",
                                                           "fc2_b", "ln1_w", "ln1_b", "ln2_w", "ln2_b"))
            need_from[l] = below
        dev = dlogits.device
        dlogits = dlogits.contiguous().float()
        nc = self.nc
        side = self._side_stream()
        # ---- head (fp32)
        dzn = torch.empty(B, 4 * D, dtype=torch.float32, device=dev)
        self._head_gemm(dlogits, prm["h3_w"], dzn, B, 4 * D, nc, nc, 4 * D, 4 * D, b_kcontig=False)
        if req["h3_w"]:
            self._wgrad(dlogits, tape.zn, gw["h3_w"], nc, 4 * D, B, nc, 4 * D, beta, side)
        if req["h3_b"]:
            self._colsum(dlogits, B, nc, nc, gw["h3_b"], beta)
        dgz = torch.empty_like(tape.gz)
        part = _ops.layernorm_bwd(dzn, tape.gz, prm["hln_w"], tape.mh, tape.rh, dgz)
        self._colsum(part[0], part.shape[1], 4 * D, 4 * D, gw["hln_w"], beta)
        self._colsum(part[1], part.shape[1], 4 * D, 4 * D, gw["hln_b"], beta)
        du = _ops.gelu_bwd(tape.u, dgz)
        dz = torch.empty(B, D, dtype=torch.float32, device=dev)
        self._head_gemm(du, prm["h0_w"], dz, B, D, 4 * D, 4 * D, D, D, b_kcontig=False)
        if req["h0_w"]:
            self._wgrad(du, tape.z, gw["h0_w"], 4 * D, D, B, 4 * D, D, beta, side)
        if req["h0_b"]:
            self._colsum(du, B, 4 * D, 4 * D, gw["h0_b"], beta)
        self._bucket_ready(self.head_range, side)
        if not need_from[L - 1]:
            if side is not None:
                torch.cuda.current_stream(dev).wait_stream(side)      # the head's weight gradients are in G
            self._finish_buckets()
            self._attach_pending()
            return None
        # ---- d(encoder output): only token-0 rows are nonzero.  Pruned (see forward): the last block's FFN / proj
        # backward runs on those B rows; otherwise on all M rows, zero outside them.
        pruned = tape.pruned
        R0 = B if pruned else M
        dx = (torch.empty if pruned else torch.zeros)(R0, D, dtype=dt, device=dev)
        _ops.copy2d(dz, D, dx, D if pruned else T * D, B, D)
        # Dropout backward as a bare mask (exact in bf16); its 1/(1-p) goes into every consumer of the masked gradient
        # (GEMM alpha, column-sum alpha, the LN kernels' bias-gradient sums) instead of a rounding of its own.  The
        # keep bits are the ones the forward's GEMM epilogues saved (mask4), not a re-hash (block_backward).
        if tape.training:
            g1 = _ops.mask4_apply(dx, torch.empty_like(dx), tape.blocks[L - 1][15], 1.0)
        else:
            g1 = dx
        g1_summed = False          # block L-1's fc2 bias gradient: g1 comes from the head (plain column sum below)
        for l in reversed(range(L)):
            if not need_from[l]:
                break
            prev_mask = tape.blocks[l - 1][15] if (tape.training and l > 0) else None
            dx, g1n = self.block_backward(l, tape.blocks[l], dx, g1, g1_summed, beta, req, side, tape.training, B,
                                          pruned and l == L - 1, chain_prev=l > 0, prev_mask=prev_mask,
                                          row0=tape.row0 and l == L - 1)
            g1_summed = l > 0
            self._bucket_ready(self.block_range[l], side)
            g1 = g1n if g1n is not None else dx
        dimg = None
        if need_from[0]:
            # ---- embedding (vit.py:39-42): dx = d(x0) [B*T, D]
            if req["cls"]:
                _ops.copy2d(dx[N:], T * D, gw["cls"].view(B, D), D, B, D, beta=beta)       # CLS row of every image
            if req["pos"]:
                self._colsum(dx, B, T * D, T * D, gw["pos"].view(-1), beta)                 # pos: sum over the batch
            dpatch = torch.empty(B * N, D, dtype=dt, device=dev)
            _ops.copy2d(dx, D, dpatch, D, B * N, D, group=(N, T))
            if req["conv_b"]:
                self._colsum(dpatch, B * N, D, D, gw["conv_b"], beta)
            if req["conv_w"]:
                self._wgrad(dpatch, tape.cols, gw["conv_w"], D, self.CPP, B * N, D, self.CPP, beta, side,
                            "gemm_wgrad")
            if tape.x_grad:                   # input-image gradient: conv dgrad = dpatch W, scattered back (col2im)
                dcols = torch.empty(B * N, self.CPP, dtype=dt, device=dev)
                _ops.gemm(dpatch, self.ww["conv_w"], dcols, B * N, self.CPP, D, D, self.CPP, self.CPP,
                          b_kcontig=False)
                dimg = torch.empty(tape.x_shape, dtype=tape.x_dtype, device=dev)
                _ops.col2im(dcols, dimg, self.P)
        self._bucket_ready(self.embed_range, side)
        if side is not None:
            torch.cuda.current_stream(dev).wait_stream(side)      # every weight gradient is in G before the step
        self._finish_buckets()
        self._attach_pending()
        return dimg

    def block_backward(self, l, saved, dx, g1, g1_summed, beta, req, side, training, B, pr=False, chain_prev=False,
                       prev_mask=None, row0=None):
        """Backward of block l from d(x_out) = dx and g1 = the fc2-dropout-masked dx (dx itself in eval).  Writes the
        block's weight gradients into the flat buffer (beta: 0 overwrite / 1 accumulate; req: which regions want a
        gradient) and returns (dx_in, g1n).  `chain_prev`: there is a block l-1 below, so the ln1 backward also emits
        block l-1's fc2 bias-gradient column sums and — in training, from its keep bits `prev_mask` — g1n, the next
        block's masked gradient (None otherwise).  `g1_summed`: this block's fc2 bias gradient was already summed by
        the block above.  `pr`: the pruned last block (dx / g1 are its B token-0 rows).  `row0`: its forward ran the
        query-0 attention (Tape.row0; None: pr and self.row0_attention, for direct callers)."""
        if row0 is None:
            row0 = pr and self.row0_attention
        D, T, H, hd, dt = self.D, self.T, self.H, self.hd, self.dtype
        M = B * T
        gw = self.gw
        prm = self.params
        es = 2 if dt == torch.bfloat16 else 4
        mk = self._mark
        dev = dx.device
        gs = 1.0 / (1.0 - DROPOUT_P) if training else 1.0
        R, rs = (B, T) if pr else (M, 1)
        x_in, a1, m1, r1, qkv, o, o32, lse, x_mid, a2, m2, r2, h, hm, pm, fm = saved
        # FFN: x_out = x_mid + drop(relu(ln2(x_mid) W1^T + b1) W2^T + b2)
        if req[f"{l}.fc2_w"]:
            self._wgrad(g1, h, gw[f"{l}.fc2_w"], D, 4 * D, R, D, 4 * D, beta, side, "gemm_wgrad", alpha=gs)
        if not g1_summed:
            self._colsum(g1, R, D, D, gw[f"{l}.fc2_b"], beta, alpha=gs)
        dh = torch.empty(R, 4 * D, dtype=dt, device=dev)
        dh_part = torch.empty(_ops.colsum_part_rows(R), 4 * D, dtype=torch.float32, device=dev)
        # relu backward and the fc1 bias-gradient column sums fused into the dgrad epilogue
        mk("gemm_dgrad", 0, 2.0 * R * 4 * D * D, (R * D + 4 * D * D + 4 * R * D) * es + R * D // 2)
        self._gemm_rows(pr, g1, self.ww[f"{l}.fc2_w"], dh, R, 4 * D, D, D, 4 * D, 4 * D, b_kcontig=False, aux=hm,
                        colsum_part=dh_part, alpha=gs, shared_cus=self.shared_cus)
        mk("gemm_dgrad", 1)
        cs_jobs = [(dh_part, [gw[f"{l}.fc1_b"]], beta)]      # this block's bias / LN-affine sums: one launch below
        if req[f"{l}.fc1_w"]:
            self._wgrad(dh, a2, gw[f"{l}.fc1_w"], 4 * D, D, R, 4 * D, D, beta, side, "gemm_wgrad")
        da2 = torch.empty(R, D, dtype=dt, device=dev)
        mk("gemm_dgrad", 0, 2.0 * R * 4 * D * D, (4 * R * D + 4 * D * D + R * D) * es)
        self._gemm_rows(pr, dh, self.ww[f"{l}.fc1_w"], da2, R, D, 4 * D, 4 * D, D, D, b_kcontig=False,
                        shared_cus=self.shared_cus)
        mk("gemm_dgrad", 1)
        dx_mid = torch.empty(R, D, dtype=dt, device=dev)
        g0 = torch.empty(R, D, dtype=dt, device=dev) if training else None
        # ln2 backward + residual add + dropout backward of the MHA branch; its third partial set is the column
        # sums of g0 as stored = the proj bias gradient
        mk("ln_bwd", 0, 0.0, (3 + 1 + (g0 is not None)) * R * D * es + 8 * R + R * D // 8)
        part = _ops.layernorm_bwd(da2, x_mid, prm[f"{l}.ln2_w"], m2, r2, dx_mid, dres=dx, drop_out=g0,
                                  drop_p=DROPOUT_P, drop_mask=pm, osum=True)
        mk("ln_bwd", 1)
        cs_jobs.append((part, [gw[f"{l}.ln2_w"], gw[f"{l}.ln2_b"], gw[f"{l}.proj_b"]], beta))
        if g0 is None:
            g0 = dx_mid
        # MHA: x_mid = x_in + drop(attn(ln1(x_in)) Wp^T + bp)
        if req[f"{l}.proj_w"]:
            self._wgrad(g0, o, gw[f"{l}.proj_w"], D, D, R, D, rs * D, beta, side, "gemm_wgrad", alpha=gs)
        do = torch.empty(R, D, dtype=dt, device=dev)
        mk("gemm_dgrad", 0, 2.0 * R * D * D, (2 * R * D + D * D) * es)
        self._gemm_rows(pr, g0, self.ww[f"{l}.proj_w"], do, R, D, D, D, D, D, b_kcontig=False, alpha=gs,
                        shared_cus=self.shared_cus)
        mk("gemm_dgrad", 1)
        if pr:
            # the ln1 backward's residual gradient on all M rows (zero outside the token-0 rows)
            dxm_full = self._token_rows("dxm", M, D, dt, T, dev)
            _ops.copy2d(dx_mid, D, dxm_full, T * D, B, D)
            dx_mid = dxm_full
        if row0:
            # attention backward from the row-0 output gradients alone (the forward computed row 0 only): dQ row 0, all
            # of dK / dV; the dQ rows 1..T-1 of this buffer are never written, so they stay zero for the dgrad /
            # wgrad GEMMs below
            dqkv = self._token_rows("dqkv", M, 3 * D, dt, T, dev)
            mk("attn_bwd", 0, 10.0 * B * H * T * hd, 4 * M * D * es + 4 * B * D * es + 4 * B * H)
            _ops.attn_bwd_row0(qkv, do, D, dqkv, B, T, H, hd, self.scale)
            mk("attn_bwd", 1)
        else:
            if pr:
                # back to all M rows for the full attention backward (zero outside the token-0 rows)
                do_full = self._token_rows("do", M, D, dt, T, dev)
                _ops.copy2d(do, D, do_full, T * D, B, D)
                do = do_full
            if o32 is None and _ops.attn_bwd_uses_o32(B, T, H, hd, dt):
                # the forward chose the fused backward (no fp32 O kept) and a library option changed since: the tiled
                # backward would form delta from the bf16 O, inexact under saturated softmax
                raise RuntimeError("attention backward needs the fp32 O that this forward did not keep: the "
                                   "attn_bwd_split library option changed between forward and backward")
            # bytes: qkv, dO, dqkv (+ O and o32 for the tiled backward's delta pass)
            mk("attn_bwd", 0, 10.0 * B * H * T * T * hd, 7 * M * D * es + 4 * B * H * T + (M * D * es + 4 * M * D if o32
                                                                                          is not None else 0))
            dqkv = _ops.attn_bwd(qkv, o, do, lse, B, T, H, hd, self.scale,
                                 workspace=self._workspace(_ops.attn_bwd_workspace_bytes(B, T, H, hd, dt)), o32=o32,
                                 shared_cus=self.shared_cus)
            mk("attn_bwd", 1)
        wq = self.ww[f"{l}.qkv_w"]
        da1 = torch.empty(M, D, dtype=dt, device=dev)
        if row0:
            # dQ is zero outside the token-0 rows: the K / V part over every row, the Q part over the B token-0 rows
            # (weight gradient: its own K = B GEMM; input gradient: added onto those rows of da1 by the residual
            # epilogue, in place)
            if req[f"{l}.qkv_w"]:
                gq = gw[f"{l}.qkv_w"]
                self._wgrad(dqkv[:, D:], a1, gq[D:], 2 * D, D, M, 3 * D, D, beta, side, "gemm_wgrad")
                self._wgrad(dqkv, a1, gq[:D], D, D, B, T * 3 * D, T * D, beta, side, "gemm_wgrad")
            mk("gemm_dgrad", 0, 2.0 * M * 2 * D * D, (2 * M * D + 2 * D * D + M * D) * es)
            self._gemm_bwd(dqkv[:, D:], wq[D:], da1, M, D, 2 * D, 3 * D, D, D, b_kcontig=False)
            mk("gemm_dgrad", 1)
            mk("gemm_dgrad", 0, 2.0 * B * D * D, (3 * B * D + D * D) * es)
            self._gemm_rows(True, dqkv, wq, da1, B, D, D, T * 3 * D, D, T * D, b_kcontig=False, res=da1,
                            ldres=T * D, shared_cus=self.shared_cus)
            mk("gemm_dgrad", 1)
        else:
            if req[f"{l}.qkv_w"]:
                self._wgrad(dqkv, a1, gw[f"{l}.qkv_w"], 3 * D, D, M, 3 * D, D, beta, side, "gemm_wgrad")
            mk("gemm_dgrad", 0, 2.0 * M * 3 * D * D, (3 * M * D + 3 * D * D + M * D) * es)
            self._gemm_bwd(dqkv, wq, da1, M, D, 3 * D, 3 * D, D, D, b_kcontig=False)
            mk("gemm_dgrad", 1)
        dx_in = torch.empty(M, D, dtype=dt, device=dev)
        g1n = torch.empty(M, D, dtype=dt, device=dev) if (training and chain_prev) else None
        # ln1 backward; for l > 0 its third partial set is the column sums of the next g1 (g1n, or dx_in in eval)
        # = the fc2 bias gradient of block l-1
        mk("ln_bwd", 0, 0.0, (3 + 1 + (g1n is not None)) * M * D * es + 8 * M)
        part = _ops.layernorm_bwd(da1, x_in, prm[f"{l}.ln1_w"], m1, r1, dx_in, dres=dx_mid, drop_out=g1n,
                                  drop_p=DROPOUT_P, drop_mask=prev_mask if g1n is not None else None,
                                  osum=chain_prev)
        mk("ln_bwd", 1)
        outs = [gw[f"{l}.ln1_w"], gw[f"{l}.ln1_b"]] + ([gw[f"{l - 1}.fc2_b"]] if chain_prev else [])
        cs_jobs.append((part, outs, beta))
        if side is not None:
            # the partial sums are finished beside the dgrad chain too: only the bucket / optimizer read the results
            side.wait_stream(torch.cuda.current_stream(self.device))
            _ops.colsum_finish_batch(cs_jobs, stream=side)
            for job in cs_jobs:
                job[0].record_stream(side)
        else:
            _ops.colsum_finish_batch(cs_jobs)
        return dx_in, g1n

    def run_param_hooks(self):
        """Parameter hooks after the fused backward (autograd's AccumulateGrad never runs for these parameters):
        `register_hook` hooks see this backward's gradient and may replace it, then
        `register_post_accumulate_grad_hook` hooks run on the parameter — each once per backward, in registration
        order.  When the backward accumulated into existing gradients, the buffer holds the increment here
        (backward() set `_acc_old`): the hooks see the increment, then the previous gradients are added back."""
        old = getattr(self, "_acc_old", None)
        self._acc_old = None
        for gv, keep in getattr(self, "_frozen_keep", None) or ():
            gv.copy_(keep)
        self._frozen_keep = None
        for p, gv in self.grad_views:
            if not p.requires_grad or p.grad is None:
                continue
            pre = p._backward_hooks
            if pre:
                g = p.grad
                for fn in pre.values():
                    r = fn(g)
                    if r is not None:
                        g = r
                if g is not p.grad:
                    p.grad.copy_(g)
        if old is not None:
            # the previous gradients go back under the views of the parameters this backward produced a gradient
            # for; every other view (frozen meanwhile, or in a region no kernel rewrote) gets its old value back,
            # never old + old
            for p, gv in self.grad_views:
                ov = torch.as_strided(old, gv.shape, gv.stride(), gv.storage_offset())
                if p.requires_grad and p.grad is not None and p.grad.data_ptr() == gv.data_ptr():
                    gv.add_(ov)
                else:
                    gv.copy_(ov)
        for p, gv in self.grad_views:
            if not p.requires_grad or p.grad is None:
                continue
            post = getattr(p, "_post_accumulate_grad_hooks", None)
            if post:
                for fn in post.values():
                    fn(p)


class ViTFunction(torch.autograd.Function):
    """One autograd node for the whole network; gradients land in the engine's flat buffer (param.grad views)."""

    @staticmethod
    def forward(ctx, x, anchor, engine, training, want_probs):
        logits, tape = engine.forward(x, training, save=True, want_probs=want_probs)
        tape.x_grad = ctx.needs_input_grad[0]
        ctx.engine = engine
        ctx.tape = tape
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        if ctx.tape is None:
            raise RuntimeError("VisionTransformer backward called twice on the same forward")
        dimg = ctx.engine.backward(ctx.tape, dlogits)
        ctx.tape = None
        ctx.engine.run_param_hooks()
        return dimg, None, None, None, None
