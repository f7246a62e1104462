"""TrainEngineBF16 — the PLA-GNN training step in bf16 storage with f32 accumulation
(BASELINE configs[4]: "hidden=512 bf16"; SURVEY.md §8d cfg5: "bf16 storage with f32
accumulate"). Not a configuration of the reference (fp32 only): reference-unpinned; the
step is checked against the fp32 oracle at a bf16 tolerance (tests/test_gpu_engine_bf16.py).

Same step as TrainEngine (code/train.py:197-207), same flat f32 master parameters, f32
gradients, f32 Adam (one launch) and f32 loss; what changes is the storage of every
N-row tensor and the operands of every product:
  * activations and activation gradients are bf16 (half the bytes of every SpMM gather
    and GEMM operand stream); every GEMM runs on v_mfma_f32_32x32x16_bf16 with f32
    accumulate (pg_gemm_bf16, 16x the f32 MFMA rate); the max aggregation selects bf16
    values exactly and its backward sums in f32 (pg_spmm_max_*_bf16);
  * the GEMMs read bf16 copies of the weights, written from the f32 master parameters by
    one gather-cast launch after every Adam step (pg_cast_f32_bf16) in the layouts the
    products want, including a stacked [Wself ; Wpool] so that the input gradient of a
    SAGE layer, dH = (dY Wself + dP Wpool) * leaky'(H), is ONE K = Fo + Fi product with a
    single rounding: dY and dP are stored side by side in DYP_l[N][Fo + Fi].
Widths are padded to multiples of 8 (16-B rows of bf16) instead of 4.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib, ops
from ._lib import PG_ARG_DEAD_NONE as DEAD_NONE, ptr
from .engine import LEAKY, MAX_GROUP_PARTS, NONE, RELU, TrainEngine, _Flat

BF16, F32 = _lib.PG_DTYPE_BF16, _lib.PG_DTYPE_F32
LEAKY_SLOPE = ops.LEAKY_SLOPE


class TrainEngineBF16(TrainEngine):
    WIDTH_ALIGN = 8
    # the stacked input-gradient weights as [Fi][Fo + Fi] (B^T, a row image: the A B^T
    # ping-pong kernel of pg_gemm_bf16 takes the product) instead of [Fo + Fi][Fi] (a k image)
    STACK_T = True
    # the fused liner1 + head kernel is f32 only: bf16 storage keeps liner1 as bf16 GEMMs
    FUSED_L1_HEAD = False

    # ------------------------------------------------------------------ buffers
    def _alloc_buffers(self, features: torch.Tensor) -> None:
        N, pd, dev, L = self.N, self.pd, self.device, self.L
        bf = dict(dtype=torch.bfloat16, device=dev)
        f32 = dict(dtype=torch.float32, device=dev)
        self.HM, self.Pl, self.arg, self.DYP, self.dM = [], [], [], [], []
        for l in range(L):
            Fi, Fo = pd[l], pd[l + 1]
            self.HM.append(torch.zeros(N, 2 * Fi, **bf))
            self.Pl.append(torch.zeros(N, Fi, **bf))
            self.arg.append(torch.zeros(N, Fi, dtype=self.dg.arg_dtype, device=dev))
            self.DYP.append(torch.zeros(N, Fo + Fi, **bf))  # [dY_l | dP_l]
            self.dM.append(torch.zeros(N, Fi, **bf))
        self.HM[0][:, :self.dims[0]] = features.to(dev, torch.float32).to(torch.bfloat16)
        self.A3 = torch.zeros(N, pd[-3], **bf)
        self.A4 = torch.zeros(N, pd[-2], **bf)
        self.prob = torch.zeros(N, pd[-1], **f32)
        self.loss = torch.zeros(2, **f32)
        self.dZ = torch.zeros(N, pd[-1], **f32)
        self.dZb = torch.zeros(N, pd[-1], **bf)
        self.dA4 = torch.zeros(N, pd[-2], **bf)
        self._build_weight_copies()

    def _build_weight_copies(self) -> None:
        """bf16 weight buffer + the gather map from the f32 flat parameters."""
        pd, L = self.pd, self.L
        wl = _Flat()
        for l in range(L):
            Fi, Fo = pd[l], pd[l + 1]
            wl.add(f"conv{l + 1}.Wpool", (Fi, Fi))
            wl.add(f"conv{l + 1}.Wcat", (Fo, 2 * Fi))
            if self.STACK_T:
                wl.add(f"conv{l + 1}.WstackT", (Fi, Fo + Fi))  # [Wself ; Wpool]^T
            else:
                wl.add(f"conv{l + 1}.Wstack", (Fo + Fi, Fi))  # [Wself ; Wpool]
        wl.add("liner1.W", (pd[-2], pd[-3]))
        idx = np.full(wl.size, -1, np.int64)
        flat_ids = self.flat_layout.views(torch.arange(self.flat_layout.size))  # flat index of every entry

        def put(name, rows: np.ndarray):
            o = wl.offsets[name]
            idx[o:o + rows.size] = rows.ravel()

        def ids(name, shape):
            t = flat_ids[name].numpy()
            assert t.shape == tuple(shape), (name, t.shape, shape)
            return t

        for l in range(L):
            Fi, Fo = pd[l], pd[l + 1]
            p = f"conv{l + 1}."
            wp = ids(p + "Wpool", (Fi, Fi))
            wc = ids(p + "Wcat", (Fo, 2 * Fi))
            put(p + "Wpool", wp)
            put(p + "Wcat", wc)
            stack = np.concatenate([wc[:, :Fi], wp], axis=0)
            if self.STACK_T:
                put(p + "WstackT", np.ascontiguousarray(stack.T))
            else:
                put(p + "Wstack", stack)
        put("liner1.W", ids("liner1.W", (pd[-2], pd[-3])))
        self.wb_layout = wl
        self.wb_map = torch.from_numpy(idx.astype(np.int32)).to(self.device)
        self.wb = torch.zeros(wl.size, dtype=torch.bfloat16, device=self.device)
        self.Wb = wl.views(self.wb)
        self._cast_weights()

    def _cast_weights(self) -> None:
        self._call("pg_cast_f32_bf16", ptr(self.flat), ptr(self.wb_map), self.wb.numel(), ptr(self.wb), self._s())

    def load_state_dict(self, sd) -> None:
        super().load_state_dict(sd)
        if hasattr(self, "wb"):
            self._cast_weights()

    def params_updated(self) -> None:
        """The bf16 weight copies follow the f32 master parameters."""
        self._cast_weights()

    def _alloc_workspace(self) -> None:
        N, pd, C, dev = self.N, self.pd, self.C, self.device
        L = _lib.lib()
        need = 0
        for l in range(self.L):
            Fi = pd[l]
            need = max(need, L.pg_spmm_max_fwd_workspace(self.dg.fwd.struct(self.ews), Fi, self.dg.arg_kind))
            need = max(need, L.pg_spmm_max_bwd_workspace(self.dg.bwd.struct(None), Fi))
        self._gemm_plans = {}
        for (M_, N_, K_) in self._wgrad_shapes():
            sk = int(L.pg_gemm_bf16_split_k(M_, N_, K_))
            self._gemm_plans[(M_, N_, K_)] = sk
            need = max(need, L.pg_gemm_bf16_workspace(M_, N_, K_, sk))
        self._parts = []
        if self.GROUP_WGRAD:
            # the grouped weight gradients' slabs: sized from the shapes alone
            self.gws = torch.empty(self._group_ws_bytes(L.pg_gemm_bf16_group_workspace), dtype=torch.uint8,
                                   device=dev)
        # the fused head (pg_mlp_head, run by forward()) and the standalone loss kernel
        need = max(need, L.pg_sigmoid_multi_loss_workspace(N, C), L.pg_mlp_head_workspace(N, C))
        self.ws = torch.zeros(max(int(need), 256), dtype=torch.uint8, device=dev)
        self.ws_bytes = self.ws.numel()

    # ------------------------------------------------------------------ kernels
    def _gemm(self, A, B, C, transa=False, transb=False, beta=0.0, bias=None, act=NONE, dact=None,
              rowsum=None, tag="gemm"):
        M = A.shape[1] if transa else A.shape[0]
        K = A.shape[0] if transa else A.shape[1]
        N = B.shape[0] if transb else B.shape[1]
        self._rec_gemm(A, B, C, M, N, K, beta, dact)
        obf = C.dtype == torch.bfloat16
        # weight gradients are recognised by their launch site, never by shape
        wgrad = tag.startswith("gemm.wgrad")
        if wgrad and (obf or bias is not None or act != NONE or dact is not None):
            raise ValueError(f"{tag}: a weight gradient has an f32 output and no epilogue")
        if self.GROUP_WGRAD and wgrad:
            q = _lib.PgGemmPart()
            q.transa, q.transb, q.M, q.N, q.K = int(transa), int(transb), M, N, K
            q.A, q.lda, q.B, q.ldb = ptr(A), A.stride(0), ptr(B), B.stride(0)
            q.beta, q.C, q.ldc, q.rowsum = beta, ptr(C), C.stride(0), ptr(rowsum)
            self._parts.append((q, 2.0 * M * N * K))
            return
        sk = self._gemm_plans.get((M, N, K), 1) if wgrad else 1
        ep = _lib.epilogue(bias, act, LEAKY_SLOPE, dact, rowsum)
        with self._t(tag, 2.0 * M * N * K):
            self._call("pg_gemm_bf16", int(transa), int(transb), M, N, K, 1.0, ptr(A), A.stride(0), ptr(B),
                 B.stride(0), beta, ptr(C), C.stride(0), BF16 if obf else F32, ep, sk, ptr(self.ws),
                 self.ws.numel(), self._s())

    def forward(self) -> None:
        st = self._s()
        g = self.dg.fwd.struct(self.ews)
        P, W, pd = self.P, self.Wb, self.pd
        for l in range(self.L):
            p = f"conv{l + 1}."
            Fi = pd[l]
            HM = self.HM[l]
            self._gemm(HM[:, :Fi], W[p + "Wpool"], self.Pl[l], transb=True, bias=P[p + "bpool"], act=RELU,
                       tag=f"gemm.fwd.pool.l{l + 1}")
            with self._t(f"spmm_max_fwd.l{l + 1}", self.spmm_bytes(l)):
                self._call("pg_spmm_max_fwd_bf16", g, ptr(self.Pl[l]), Fi, Fi, ptr(HM[:, Fi:]), HM.stride(0),
                     ptr(self.arg[l]), Fi, self.dg.arg_kind | DEAD_NONE, ptr(self.ws), self.ws_bytes, st)
            Fo = pd[l + 1]
            out = self.HM[l + 1][:, :Fo] if l + 1 < self.L else self.A3
            self._gemm(HM, W[p + "Wcat"], out, transb=True, bias=P[p + "b"], act=LEAKY,
                       tag=f"gemm.fwd.cat.l{l + 1}")
        self._gemm(self.A3, W["liner1.W"], self.A4, transb=True, bias=P["liner1.b"], act=LEAKY,
                   tag="gemm.fwd.liner1")
        # liner2 + loss + dZ + dA4 (f32 W2 / b2; bf16 A4, dZ copy and dA4)
        self._head(BF16, self.A4, self.dZ, self.dZb, self.dA4)

    def backward(self) -> None:
        st = self._s()
        G, P, W, pd = self.G, self.P, self.Wb, self.pd
        g = self.dg.fwd.struct(self.ews)
        gt = self.dg.bwd.struct(None)
        # liner2 / liner1 (weights W[out][in] as k images for the input gradients)
        self._gemm(self.dZb, self.A4, G["liner2.W"], transa=True, rowsum=G["liner2.b"], tag="gemm.wgrad.liner2")
        self._gemm(self.dA4, self.A3, G["liner1.W"], transa=True, rowsum=G["liner1.b"], tag="gemm.wgrad.liner1")
        top = self.L - 1
        self._gemm(self.dA4, W["liner1.W"], self.DYP[top][:, :pd[top + 1]], act=LEAKY, dact=self.A3,
                   tag="gemm.dgrad.liner1")
        for l in reversed(range(self.L)):
            p = f"conv{l + 1}."
            Fi, Fo = pd[l], pd[l + 1]
            HM, DYP = self.HM[l], self.DYP[l]
            dY, dP = DYP[:, :Fo], DYP[:, Fo:]
            self._gemm(dY, HM, G[p + "Wcat"], transa=True, rowsum=G[p + "b"], tag=f"gemm.wgrad.cat.l{l + 1}")
            # dM = dY Wneigh   (Wneigh = the right half of Wcat, read as a [Fo][Fi] k image)
            self._gemm(dY, W[p + "Wcat"][:, Fi:], self.dM[l], tag=f"gemm.dgrad.neigh.l{l + 1}")
            with self._t(f"spmm_max_bwd.l{l + 1}", self.spmm_bwd_bytes(l)):
                self._call("pg_spmm_max_bwd_bf16", g, gt, ptr(self.arg[l]), Fi, self.dg.arg_kind | DEAD_NONE, ptr(self.dM[l]),
                     Fi, Fi, ptr(self.Pl[l]), Fi, None, 0, ptr(dP), DYP.stride(0),
                     ptr(self.ws), self.ws_bytes, st)
            self._gemm(dP, HM[:, :Fi], G[p + "Wpool"], transa=True, rowsum=G[p + "bpool"],
                       tag=f"gemm.wgrad.pool.l{l + 1}")
            self._wgrad_bucket_boundary(l)
            if l > 0:
                # dH = ([dY | dP] [Wself ; Wpool]) * leaky'(H) -> the lower layer's dY
                if self.STACK_T:
                    self._gemm(DYP, W[p + "WstackT"], self.DYP[l - 1][:, :Fi], transb=True, act=LEAKY,
                               dact=HM[:, :Fi], tag=f"gemm.dgrad.stack.l{l + 1}")
                else:
                    self._gemm(DYP, W[p + "Wstack"], self.DYP[l - 1][:, :Fi], act=LEAKY, dact=HM[:, :Fi],
                               tag=f"gemm.dgrad.stack.l{l + 1}")
        self._reduce_deferred()
        self._bucket_done(len(self.grad_buckets()) - 1)

    def _reduce_deferred(self) -> None:
        """Every weight gradient of the step as one grouped split-K launch + one combine
        (pg_gemm_bf16_group): they only feed Adam, so they all wait for the backward's end."""
        parts, self._parts = self._parts, []
        for i in range(0, len(parts), MAX_GROUP_PARTS):  # the library's part limit per launch
            chunk = parts[i:i + MAX_GROUP_PARTS]
            arr = (_lib.PgGemmPart * len(chunk))(*[q for q, _ in chunk])
            with self._t("gemm.wgrad.group", sum(w for _, w in chunk)):
                self._call("pg_gemm_bf16_group", arr, len(chunk), ptr(self.gws), self.gws.numel(), self._s())

    def adam(self) -> None:
        super().adam()
        with self._t("adam"):
            self._cast_weights()

    # ------------------------------------------------------------------ accounting
    def spmm_bytes(self, layer: int) -> int:
        """SURVEY.md §8(d) B_fwd with s = 2 (bf16 features): 4(N+1) + 4E' + 2F E' + 2F N + aF N."""
        N, E, F = self.N, self.dg.num_edges, self.dims[layer]
        a = 2 if self.dg.arg_kind == _lib.PG_ARG_U16 else 4
        return 4 * (N + 1) + 4 * E + 2 * F * E + 2 * F * N + a * F * N

    def spmm_bwd_bytes(self, layer: int) -> int:
        """B_bwd with s = 2: dM, argmax, relu mask read once, dP written once, + the
        transposed CSR."""
        N, E, F = self.N, self.dg.num_edges, self.dims[layer]
        a = 2 if self.dg.arg_kind == _lib.PG_ARG_U16 else 4
        return 4 * (N + 1) + 8 * E + (6 + a) * F * N

    def logits(self) -> torch.Tensor:
        return self.prob[:, :self.C]
