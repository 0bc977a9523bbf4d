"""dct_amd -- MI355X-native 8x8 DCT + quantization hot path of erkinov-wtf/dct.

Python host over the C-ABI of ``libdct_amd.so`` (include/dct_amd.h, and the
reference's per-block API include/dct.h / include/quantization.h).  PyTorch is
used only as the owner of device memory and streams: tensors are handed to the
library as raw pointers on torch's current HIP stream, so torch.cuda.Event
timing sees the kernels.

The library is REQUIRED: importing a compute entry point without a built
``libdct_amd.so`` raises -- there is no CPU fallback in this package.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libdct_amd.so")

# synthetic frame kinds (include/dct_amd.h, dctq_synth)
KINDS = {"uniform": 0, "smooth": 1, "const": 2, "extreme": 3}


class DctqError(RuntimeError):
    pass


class _Plane(C.Structure):
    _fields_ = [("pixels", C.c_void_p), ("stride", C.c_longlong), ("frame_stride", C.c_longlong),
                ("width", C.c_int), ("height", C.c_int), ("nframes", C.c_int)]


_lib = None
_diag = None
DIAG_PATH = os.path.join(HERE, "libdct_amd_diag.so")


def _bind(L: C.CDLL, diagnostic: bool) -> C.CDLL:
    vp, i, ll = C.c_void_p, C.c_int, C.c_longlong
    sig = {
        "dctq_plan_create": ([i, i, C.POINTER(vp)], i),
        "dctq_plan_destroy": ([vp], None),
        "dctq_plan_set_fallback_counter": ([vp, vp], i),
        "dctq_forward_quant": ([vp, C.POINTER(_Plane), vp, vp, vp], i),
        "dctq_forward_quant_planes": ([vp, C.POINTER(_Plane), i, vp, vp, vp], i),
        "dctq_round_trip_planes": ([vp, C.POINTER(_Plane), i, vp, vp, vp, vp], i),
        "dctq_encode_workspace_bytes": ([ll], C.c_size_t),
        "dctq_encode_planes": ([vp, C.POINTER(_Plane), i, vp, vp, vp, ll, vp, vp], i),
        "dctq_encode_planes16": ([vp, C.POINTER(_Plane), i, vp, vp, vp, ll, vp, vp], i),
        "dctq_abi_version": ([], i),
        "dctq_forward_float": ([vp, C.POINTER(_Plane), vp, vp], i),
        "dctq_inverse": ([vp, vp, vp, ll, vp, vp], i),
        "dctq_synth": ([C.c_uint64, i, C.POINTER(_Plane), vp], i),
        "dctq_error_string": ([i], C.c_char_p),
        "dctq_synchronize": ([vp], i),
        "dctq_rle_workspace_bytes": ([ll], C.c_size_t),
        "dctq_rle_count": ([vp, ll, vp, vp, vp], i),
        "dctq_rle_emit": ([vp, ll, vp, vp, vp], i),
        "dctq_rle_decode": ([vp, vp, ll, vp, vp], i),
        "dctq_rle_decode16": ([vp, vp, ll, vp, vp], i),
        "dctq_plan_symbol_bytes": ([vp], i),
        "dctq_huffman_bits": ([vp, ll, vp, vp], i),
        "dctq_huffman_bits_planes": ([vp, C.POINTER(_Plane), i, vp, vp], i),
        "dctq_stream_release": ([vp], i),
    }
    if diagnostic:
        sig.update({
            "dctq_diag_plan_set_variant": ([vp, i], i),
            "dctq_diag_forward_quant_planes": ([vp, C.POINTER(_Plane), i, vp, vp, vp], i),
            "dctq_diag_forward_float": ([vp, C.POINTER(_Plane), vp, vp], i),
            "dctq_diag_inverse": ([vp, vp, vp, ll, vp, vp], i),
            "dctq_diag_plan_set_num_cus": ([vp, i], i),
            "dctq_diag_plan_set_inverse": ([vp, i], i),
            "dctq_debug_inverse_bound": ([i, i, C.POINTER(i)], C.c_double),
            "dctq_debug_symbol_bytes": ([i, i], i),
            "dctq_diag_legacy_lanes": ([C.POINTER(i), C.POINTER(i)], i),
            "dctq_diag_movement_planes": ([vp, C.POINTER(_Plane), i, vp, vp], i),
            "dctq_diag_movement_v2_planes": ([vp, C.POINTER(_Plane), i, vp, vp], i),
            "dctq_diag_movement_grid_planes": ([vp, C.POINTER(_Plane), i, vp, i, vp], i),
            "dctq_diag_rt_movement_planes": ([vp, C.POINTER(_Plane), i, vp, vp, vp], i),
            "dctq_diag_stream": ([i, vp, vp, ll, vp], i),
            "dctq_diag_stream_release": ([vp], i),
            "dctq_debug_tables": ([i, i, vp, vp, vp, vp], i),
            "dctq_debug_fastdiv": ([C.c_uint32, C.c_uint32], i),
            "dctq_debug_dc_table": ([i, vp], i),
            "dctq_debug_forward_kernel": ([i, i, ll, i], i),
            "dctq_diag_stream_stash_bytes": ([vp], ll),
        })
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    return L


def lib() -> C.CDLL:
    """Load libdct_amd.so, the product library (fails loudly if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise DctqError(f"{LIB_PATH} is missing: run `python -m dct_amd.build` (hipcc, gfx950)")
        _lib = _bind(C.CDLL(LIB_PATH), False)
    return _lib


def diag() -> C.CDLL:
    """Load libdct_amd_diag.so: the same kernels plus the diagnostic entry points of
    csrc/dctq_diag.h (test-only kernel selection, movement / hardware ceilings, host
    table introspection).  Never used by the product path."""
    global _diag
    if _diag is None:
        if not os.path.exists(DIAG_PATH):
            raise DctqError(f"{DIAG_PATH} is missing: run `python -m dct_amd.build` (hipcc, gfx950)")
        _diag = _bind(C.CDLL(DIAG_PATH), True)
    return _diag


def _check(rc: int, L: C.CDLL = None) -> None:
    if rc != 0:
        raise DctqError(f"dctq error {rc}: {(L or lib()).dctq_error_string(rc).decode()}")


def _need(t, numel: int, dtype, what: str, device=None):
    """A caller-supplied buffer must be a contiguous device tensor of the right
    dtype holding at least `numel` elements (on `device` when given): the kernels
    write through the raw pointer, so a short or host tensor is refused here."""
    import torch
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise DctqError(f"{what} must be a tensor on a HIP device")
    if t.dtype != dtype:
        raise DctqError(f"{what} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise DctqError(f"{what} must be contiguous")
    if t.numel() < numel:
        raise DctqError(f"{what} holds {t.numel()} elements, {numel} needed")
    if device is not None and t.device != device:
        raise DctqError(f"{what} is on {t.device}, the input is on {device}")
    return t


def _stream_ptr(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


def plane_desc(px, width: int = None, height: int = None):
    """Describe a uint8 CUDA tensor [H, W] or [F, H, W] (rows may be padded: stride = px.stride(-2))."""
    import torch
    if px.dtype != torch.uint8 or not px.is_cuda:
        raise DctqError("pixels must be a uint8 tensor on a HIP device")
    if px.dim() == 2:
        px = px.unsqueeze(0)
    if px.dim() != 3 or px.stride(-1) != 1:
        raise DctqError("pixels must be [H, W] or [F, H, W] with unit column stride")
    f, h, w = px.shape
    return _Plane(px.data_ptr(), px.stride(1), px.stride(0) if f > 1 else px.stride(1) * h,
                  width if width is not None else w, height if height is not None else h, f)


def _need_planes(outs, var_nums, recons, nbs, planes):
    """Per-plane output lists of the multi-plane calls: one entry per plane, each
    sized for that plane's blocks (_need)."""
    import torch
    for name, ts, per, dt in (("outs", outs, 64, torch.int16), ("var_nums", var_nums, 1, torch.int32),
                              ("recons", recons, 64, torch.float32)):
        if ts is None:
            continue
        if len(ts) != len(nbs):
            raise DctqError(f"{name} needs one tensor per plane ({len(nbs)}), got {len(ts)}")
        for k, (t, nb, px) in enumerate(zip(ts, nbs, planes)):
            _need(t, nb * per, dt, f"{name}[{k}]", px.device)


class Plan:
    """Tables for one (quality, adaptive) configuration on the current device
    (quant_init(8, quality, adaptive) semantics, src/quantization.c:19-41)."""

    def __init__(self, quality: int = 50, adaptive: bool = False, variant: int = None, diagnostic: bool = False,
                 num_cus: int = None, inverse: str = None):
        """variant (tests / A/B only): force the forward kernel through the diagnostic
        library (dctq_diag_plan_set_variant: 1 = v1, 3 = v3 in-place ties, 4 = v2 tie
        queue, at any size); num_cus (tests only): launch as if the device had that many
        CUs (dctq_diag_plan_set_num_cus: smaller grids, more batches per wave);
        diagnostic: create the plan in the diagnostic library (needed for
        diag_movement_planes); inverse="fp64" (tests only): the fused round trip uses
        the paired-lane fp64 inverse even when the plan is admitted to the fp32 one
        (dctq_diag_plan_set_inverse)."""
        self.quality, self.adaptive = quality, bool(adaptive)
        diagnostic = diagnostic or variant is not None or num_cus is not None or inverse is not None
        self._L = diag() if diagnostic else lib()
        # a forced variant is honoured by the diagnostic entry points only (csrc/dctq_diag.h)
        self._diag = variant is not None
        h = C.c_void_p()
        self._chk(self._L.dctq_plan_create(int(quality), int(bool(adaptive)), C.byref(h)))
        self._h = h
        if variant is not None:
            self._chk(self._L.dctq_diag_plan_set_variant(h, int(variant)))
        if num_cus is not None:
            self._chk(self._L.dctq_diag_plan_set_num_cus(h, int(num_cus)))
        if inverse is not None:
            if inverse not in ("fp64", "auto"):
                raise DctqError('inverse must be "fp64" or "auto"')
            self._chk(self._L.dctq_diag_plan_set_inverse(h, 0 if inverse == "fp64" else 1))

    def _chk(self, rc: int) -> None:
        _check(rc, self._L)

    def close(self):
        if getattr(self, "_h", None):
            self._L.dctq_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_fallback_counter(self, counter):
        """counter: int64 CUDA tensor of one element (or None)."""
        self._chk(self._L.dctq_plan_set_fallback_counter(self._h, C.c_void_p(counter.data_ptr()) if counter is not None else None))

    # --- hot path -------------------------------------------------------
    def forward_quant(self, px, out=None, var_num=None, stream=None):
        """u8 [H,W] / [F,H,W] -> int16 [F*H/8*W/8, 64] quantized coefficients (bit-exact)."""
        import torch
        d = plane_desc(px)
        nblk = d.nframes * (d.width // 8) * (d.height // 8)
        if out is None:
            out = torch.empty((nblk, 64), dtype=torch.int16, device=px.device)
        _need(out, nblk * 64, torch.int16, "out", px.device)
        if var_num is not None:
            _need(var_num, nblk, torch.int32, "var_num", px.device)
        vn = C.c_void_p(var_num.data_ptr()) if var_num is not None else None
        if self._diag:
            op, vp = (C.c_void_p * 1)(out.data_ptr()), (C.c_void_p * 1)(vn.value) if vn is not None else None
            self._chk(self._L.dctq_diag_forward_quant_planes(self._h, C.byref(d), 1, C.cast(op, C.c_void_p),
                                                             C.cast(vp, C.c_void_p) if vp is not None else None,
                                                             _stream_ptr(stream)))
        else:
            self._chk(self._L.dctq_forward_quant(self._h, C.byref(d), C.c_void_p(out.data_ptr()), vn,
                                                 _stream_ptr(stream)))
        return out

    def forward_quant_planes(self, planes, outs=None, var_nums=None, stream=None):
        """Up to 4 u8 planes of any geometry (e.g. Y, Cb, Cr) in ONE launch; returns the list
        of int16 [nblk_k, 64] outputs, each equal to forward_quant(planes[k])."""
        import torch
        n = len(planes)
        descs = (_Plane * n)(*[plane_desc(px) for px in planes])
        nbs = [d.nframes * (d.width // 8) * (d.height // 8) for d in descs]
        if outs is None:
            outs = [torch.empty((nb, 64), dtype=torch.int16, device=px.device) for nb, px in zip(nbs, planes)]
        _need_planes(outs, var_nums, None, nbs, planes)
        cp = (C.c_void_p * n)(*[o.data_ptr() for o in outs])
        vp = (C.c_void_p * n)(*[v.data_ptr() for v in var_nums]) if var_nums is not None else None
        fn = self._L.dctq_diag_forward_quant_planes if self._diag else self._L.dctq_forward_quant_planes
        self._chk(fn(self._h, descs, n, C.cast(cp, C.c_void_p), C.cast(vp, C.c_void_p) if vp is not None else None,
                     _stream_ptr(stream)))
        return outs

    def diag_movement_planes(self, planes, outs, stream=None, shape: int = 3, grid_mult: int = 0):
        """DIAGNOSTIC: the bytes forward_quant_planes moves, with no arithmetic (outs receive
        pixel bytes, not coefficients) -- the memory ceiling of that access pattern."""
        n = len(planes)
        descs = (_Plane * n)(*[plane_desc(px) for px in planes])
        _need_planes(outs, None, None, [d.nframes * (d.width // 8) * (d.height // 8) for d in descs], planes)
        cp = (C.c_void_p * n)(*[o.data_ptr() for o in outs])
        if self._L is not _diag:
            raise DctqError("diag_movement_planes needs a plan of the diagnostic library (Plan(..., diagnostic=True))")
        if grid_mult:
            self._chk(self._L.dctq_diag_movement_grid_planes(self._h, descs, n, C.cast(cp, C.c_void_p), grid_mult,
                                                             _stream_ptr(stream)))
            return outs
        fn = self._L.dctq_diag_movement_planes if shape == 3 else self._L.dctq_diag_movement_v2_planes
        self._chk(fn(self._h, descs, n, C.cast(cp, C.c_void_p), _stream_ptr(stream)))
        return outs

    def diag_rt_movement_planes(self, planes, outs, recons, stream=None):
        """DIAGNOSTIC: the bytes round_trip_planes moves (its grid, stage and stores), with no
        arithmetic (outs/recons receive pixel bytes) -- the memory ceiling of that pattern."""
        n = len(planes)
        descs = (_Plane * n)(*[plane_desc(px) for px in planes])
        nbs = [d.nframes * (d.width // 8) * (d.height // 8) for d in descs]
        _need_planes(outs, None, recons, nbs, planes)
        if self._L is not _diag:
            raise DctqError("diag_rt_movement_planes needs a plan of the diagnostic library (Plan(..., diagnostic=True))")
        cp = (C.c_void_p * n)(*[o.data_ptr() for o in outs])
        rp = (C.c_void_p * n)(*[r.data_ptr() for r in recons])
        self._chk(self._L.dctq_diag_rt_movement_planes(self._h, descs, n, C.cast(cp, C.c_void_p), C.cast(rp, C.c_void_p),
                                                      _stream_ptr(stream)))
        return outs, recons

    def round_trip_planes(self, planes, outs=None, recons=None, var_nums=None, stream=None):
        """Fused forward + inverse of up to 4 planes in ONE launch.  Returns (coefs, recons):
        int16 [nblk_k, 64] (== forward_quant) and float32 [nblk_k, 64]
        (== inverse(coef, var_num) within 1e-4)."""
        import torch
        n = len(planes)
        descs = (_Plane * n)(*[plane_desc(px) for px in planes])
        nbs = [d.nframes * (d.width // 8) * (d.height // 8) for d in descs]
        if outs is None:
            outs = [torch.empty((nb, 64), dtype=torch.int16, device=px.device) for nb, px in zip(nbs, planes)]
        if recons is None:
            recons = [torch.empty((nb, 64), dtype=torch.float32, device=px.device) for nb, px in zip(nbs, planes)]
        _need_planes(outs, var_nums, recons, nbs, planes)
        cp = (C.c_void_p * n)(*[o.data_ptr() for o in outs])
        rp = (C.c_void_p * n)(*[r.data_ptr() for r in recons])
        vp = (C.c_void_p * n)(*[v.data_ptr() for v in var_nums]) if var_nums is not None else None
        self._chk(self._L.dctq_round_trip_planes(self._h, descs, n, C.cast(cp, C.c_void_p),
                                            C.cast(vp, C.c_void_p) if vp is not None else None,
                                            C.cast(rp, C.c_void_p), _stream_ptr(stream)))
        return outs, recons

    @property
    def symbol_bytes(self) -> int:
        """The most compact symbol format this plan admits (dctq_plan_symbol_bytes): 2 when the
        plan bounds every |quantized coefficient| by 511 (dctq_encode_planes16), else 4."""
        return int(self._L.dctq_plan_symbol_bytes(self._h))

    def encode_planes(self, planes, outs=None, capacity=None, stream=None, symbol_bytes=None):
        """Forward + zigzag/RLE of up to 4 planes (the count fused into the forward launch).
        Returns (coefs [int16 [nblk_k, 64]], offsets int32 [N+1], symbols [total]) -- offsets
        hold uint32 bit patterns, blocks numbered plane by plane.  symbol_bytes 4
        (dctq_encode_planes): int32 holding (uint16)value | run << 16; 2
        (dctq_encode_planes16, only where the plan admits it): int16 holding
        run << 10 | (value & 0x3FF); None: the most compact format the plan admits
        (self.symbol_bytes).  capacity (symbols) defaults to the worst case (64 per block).
        Reads the total back (one sync)."""
        import torch
        sb = self.symbol_bytes if symbol_bytes is None else int(symbol_bytes)
        if sb not in (2, 4):
            raise ValueError("symbol_bytes must be 2 or 4")
        n = len(planes)
        descs = (_Plane * n)(*[plane_desc(px) for px in planes])
        nbs = [d.nframes * (d.width // 8) * (d.height // 8) for d in descs]
        nb = sum(nbs)
        dev = planes[0].device
        if outs is None:
            outs = [torch.empty((m, 64), dtype=torch.int16, device=dev) for m in nbs]
        _need_planes(outs, None, None, nbs, planes)
        cap = 64 * nb if capacity is None else int(capacity)
        off = torch.empty(nb + 1, dtype=torch.int32, device=dev)
        sym = torch.empty(max(cap, 1), dtype=torch.int16 if sb == 2 else torch.int32, device=dev)
        ws = torch.empty(int(self._L.dctq_encode_workspace_bytes(nb)) // 4 + 1, dtype=torch.int32, device=dev)
        cp = (C.c_void_p * n)(*[o.data_ptr() for o in outs])
        fn = self._L.dctq_encode_planes16 if sb == 2 else self._L.dctq_encode_planes
        self._chk(fn(self._h, descs, n, C.cast(cp, C.c_void_p), C.c_void_p(off.data_ptr()),
                     C.c_void_p(sym.data_ptr()), cap, C.c_void_p(ws.data_ptr()), _stream_ptr(stream)))
        total = int(off[nb].item()) & 0xFFFFFFFF
        return outs, off, sym[:min(total, cap)]

    def huffman_bits_planes(self, planes, out=None, stream=None):
        """Per-block Huffman size straight from up to 4 u8 planes (the whole per-block loop of
        tests/test_entropy.c:300-341 on the GPU, coefficients kept on chip): int32 [N], blocks
        numbered plane by plane, equal to huffman_bits(cat(forward_quant_planes(planes)))."""
        import torch
        n = len(planes)
        descs = (_Plane * n)(*[plane_desc(px) for px in planes])
        nb = sum(d.nframes * (d.width // 8) * (d.height // 8) for d in descs)
        if out is None:
            out = torch.empty(nb, dtype=torch.int32, device=planes[0].device)
        _need(out, nb, torch.int32, "out", planes[0].device)
        self._chk(self._L.dctq_huffman_bits_planes(self._h, descs, n, C.c_void_p(out.data_ptr()),
                                                   _stream_ptr(stream)))
        return out

    def forward_float(self, px, out=None, stream=None):
        import torch
        d = plane_desc(px)
        nblk = d.nframes * (d.width // 8) * (d.height // 8)
        if out is None:
            out = torch.empty((nblk, 64), dtype=torch.float32, device=px.device)
        _need(out, nblk * 64, torch.float32, "out", px.device)
        fn = self._L.dctq_diag_forward_float if self._diag else self._L.dctq_forward_float
        self._chk(fn(self._h, C.byref(d), C.c_void_p(out.data_ptr()), _stream_ptr(stream)))
        return out

    def inverse(self, coef, var_num=None, out=None, stream=None):
        """int16 [N, 64] -> float32 [N, 64] = dct_inverse(dequantize(coef)) + 128."""
        import torch
        _need(coef, 0, torch.int16, "coef")
        n = coef.numel() // 64
        if out is None:
            out = torch.empty((n, 64), dtype=torch.float32, device=coef.device)
        _need(out, n * 64, torch.float32, "out", coef.device)
        if var_num is not None:
            _need(var_num, n, torch.int32, "var_num", coef.device)
        fn = self._L.dctq_diag_inverse if self._diag else self._L.dctq_inverse
        self._chk(fn(self._h, C.c_void_p(coef.data_ptr()), C.c_void_p(var_num.data_ptr()) if var_num is not None else None,
                     n, C.c_void_p(out.data_ptr()), _stream_ptr(stream)))
        return out


def stream_release(stream=None, diagnostic: bool = False) -> None:
    """diagnostic=True: dctq_diag_stream_release -- wait for `stream` (torch's current
    one by default) and free the tie-path stashes this thread's v2 (variant 4)
    launches on it hold.  The product's dctq_stream_release is a no-op (it keeps no
    per-stream memory)."""
    L = diag() if diagnostic else lib()
    fn = L.dctq_diag_stream_release if diagnostic else L.dctq_stream_release
    _check(fn(_stream_ptr(stream)), L)


def rle_encode(coef, stream=None):
    """Zigzag + run-length symbols of int16 blocks [N, 64] (src/entropy.c run_length_encode per
    block, concatenated).  Returns (offsets [N+1], symbols [total]) as int32 tensors holding the
    uint32 bit patterns: symbol = (uint16)value | run << 16.  Reads the total back (one sync)."""
    import torch
    _need(coef, 0, torch.int16, "coef")
    n = coef.numel() // 64
    ws = torch.empty(int(lib().dctq_rle_workspace_bytes(n)) // 4 + 1, dtype=torch.int32, device=coef.device)
    off = torch.empty(n + 1, dtype=torch.int32, device=coef.device)
    s = _stream_ptr(stream)
    _check(lib().dctq_rle_count(C.c_void_p(coef.data_ptr()), n, C.c_void_p(off.data_ptr()),
                                C.c_void_p(ws.data_ptr()), s))
    total = int(off[n].item()) & 0xFFFFFFFF
    sym = torch.empty(max(total, 1), dtype=torch.int32, device=coef.device)
    _check(lib().dctq_rle_emit(C.c_void_p(coef.data_ptr()), n, C.c_void_p(off.data_ptr()),
                               C.c_void_p(sym.data_ptr()), s))
    return off, sym[:total]


def huffman_bits(coef, out=None, stream=None):
    """int16 [N, 64] quantized blocks -> int32 [N]: per block, the bits the reference's
    get_encoded_size reports after build_huffman_codes on that block's RLE symbols
    (tests/test_entropy.c:329-341)."""
    import torch
    _need(coef, 0, torch.int16, "coef")
    n = coef.numel() // 64
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=coef.device)
    _need(out, n, torch.int32, "out", coef.device)
    _check(lib().dctq_huffman_bits(C.c_void_p(coef.data_ptr()), n, C.c_void_p(out.data_ptr()), _stream_ptr(stream)))
    return out


def rle_decode(symbols, offsets, out=None, stream=None):
    """Inverse of rle_encode / encode_planes: int16 [N, 64] blocks (run_length_decode +
    zigzag_to_block).  int16 symbols are the 2-byte format (dctq_rle_decode16)."""
    import torch
    n = offsets.numel() - 1
    if out is None:
        out = torch.empty((n, 64), dtype=torch.int16, device=offsets.device)
    _need(out, n * 64, torch.int16, "out", offsets.device)
    fn = lib().dctq_rle_decode16 if symbols.dtype == torch.int16 else lib().dctq_rle_decode
    _check(fn(C.c_void_p(symbols.data_ptr()), C.c_void_p(offsets.data_ptr()), n, C.c_void_p(out.data_ptr()),
              _stream_ptr(stream)))
    return out


def symbol_bytes(quality: int, adaptive: bool = False) -> int:
    """Host-only: the encoder's symbol format of a standard-table plan (2 or 4 bytes)."""
    return int(diag().dctq_debug_symbol_bytes(int(quality), int(bool(adaptive))))


def synth(seed: int, kind, width: int, height: int, nframes: int = 1, device="cuda", stream=None, out=None):
    """Synthetic u8 frames [F, H, W] generated on the device (oracle-identical)."""
    import torch
    k = KINDS[kind] if isinstance(kind, str) else int(kind)
    if out is None:
        out = torch.empty((nframes, height, width), dtype=torch.uint8, device=device)
    d = plane_desc(out)
    _check(lib().dctq_synth(C.c_uint64(seed), k, C.byref(d), _stream_ptr(stream)))
    return out


def forward_kernel(quality: int, adaptive: bool, batches: int, num_cus: int) -> str:
    """Name of the forward kernel dctq_forward_quant_planes launches for this plan over
    `batches` 64-block batches on num_cus CUs (host-only, dctq_debug_forward_kernel)."""
    v = diag().dctq_debug_forward_kernel(int(quality), int(bool(adaptive)), int(batches), int(num_cus))
    return f"fdct8_quant_v{v}<{str(bool(adaptive)).lower()}, false, false>"


def inverse_bound(quality: int, adaptive: bool = False):
    """Host-only: (bound, admitted) -- the rigorous bound of |recon - reference| of the
    fused round trip's fp32 inverse for this standard-table plan, and whether
    round_trip_planes runs that inverse for it (tools/inv_bound.py, api.hip)."""
    a = C.c_int(0)
    b = diag().dctq_debug_inverse_bound(int(quality), int(bool(adaptive)), C.byref(a))
    return float(b), bool(a.value)


def debug_tables(quality: int, adaptive: bool = False):
    """Host-only: the (w, thr, D, Q) tables a plan would upload (no GPU needed)."""
    import numpy as np
    w = np.zeros(64, np.float32)
    thr = np.zeros(64, np.float32)
    d = np.zeros(64, np.float64)
    q = np.zeros(64, np.float64)
    _check(diag().dctq_debug_tables(quality, int(adaptive), w.ctypes.data, thr.ctypes.data, d.ctypes.data,
                                    q.ctypes.data))
    return w, thr, d, q
