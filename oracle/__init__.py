"""oracle -- TEST INFRASTRUCTURE ONLY (parity checker and CPU baseline).

ctypes wrappers over

* ``liboracle.so``   -- the clean-room C restatement (``dct_oracle.c``) that
  follows the reference's operation order bit for bit, and
* ``_ref/libref.so`` -- the reference's own ``src/{utils,dct,quantization,entropy}.c``
  compiled from ``/root/reference`` by ``oracle/Makefile`` (present when it was
  built in the container; it travels to the GPU box with the snapshot).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg may import this package.  The product (``dct_amd``) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_ORC = os.path.join(HERE, "liboracle.so")
_REF = os.path.join(HERE, "_ref", "libref.so")

_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_ip = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_i16p = np.ctypeslib.ndpointer(dtype=np.int16, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")


def build(quiet: bool = True) -> None:
    """Compile liboracle.so (and _ref/libref.so when /root/reference exists)."""
    out = subprocess.run(["make", "-C", HERE], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)
    if not quiet:
        print(out.stdout)


def _load_orc():
    if not os.path.exists(_ORC):
        build()
    lib = C.CDLL(_ORC)
    lib.orc_dct_matrix.argtypes = [C.c_int, _dp]
    lib.orc_quant_matrix.argtypes = [C.c_int, C.c_int, _dp]
    lib.orc_dequant_matrix.argtypes = [C.c_int, _dp, _dp]
    lib.orc_clamp_quality.argtypes = [C.c_int]
    lib.orc_clamp_quality.restype = C.c_int
    lib.orc_forward.argtypes = [C.c_int, _dp, _dp, _dp]
    lib.orc_inverse.argtypes = [C.c_int, _dp, _dp, _dp]
    lib.orc_forward_tables.argtypes = [C.c_int, _dp, _dp, _dp, _dp]
    lib.orc_inverse_tables.argtypes = [C.c_int, _dp, _dp, _dp, _dp]
    lib.orc_variance.argtypes = [C.c_int, _dp]
    lib.orc_variance.restype = C.c_double
    lib.orc_adjust.argtypes = [C.c_int, _dp, C.c_double, C.c_int, _dp]
    lib.orc_quantize.argtypes = [C.c_int, _dp, C.c_int, C.c_double, _dp, _ip]
    lib.orc_dequantize.argtypes = [C.c_int, _dp, C.c_int, C.c_double, _ip, _dp]
    lib.orc_forward_plane.argtypes = [_u8p, C.c_long, C.c_int, C.c_int, C.c_int, C.c_int,
                                      C.c_void_p, C.c_void_p, C.c_int]
    lib.orc_inverse_plane.argtypes = [_i16p, C.c_void_p, C.c_int, C.c_int, C.c_int, _dp]
    lib.orc_plane_variance.argtypes = [_u8p, C.c_long, C.c_int, C.c_int, _dp]
    lib.orc_splitmix.argtypes = [C.c_uint64, C.c_uint64]
    lib.orc_splitmix.restype = C.c_uint64
    lib.orc_synth_plane.argtypes = [C.c_uint64, C.c_int, C.c_int, C.c_int, _u8p, C.c_long]
    lib.orc_zigzag_order.argtypes = [C.c_int, _ip]
    lib.orc_rle_encode.argtypes = [C.c_int, _ip, _ip, _ip]
    lib.orc_rle_decode.argtypes = [C.c_int, _ip, _ip, C.c_int, _ip]
    lib.orc_rle_encode_plane.argtypes = [_i16p, C.c_long, C.c_void_p, C.c_void_p]
    lib.orc_rle_encode_plane.restype = C.c_long
    lib.orc_huffman_bits.argtypes = [_ip]
    lib.orc_huffman_bits.restype = C.c_int
    lib.orc_huffman_bits_plane.argtypes = [_i16p, C.c_long, C.c_void_p]
    return lib


_orc = None


def orc():
    global _orc
    if _orc is None:
        _orc = _load_orc()
    return _orc


def ref_available() -> bool:
    return os.path.exists(_REF)


_refs = {}


def ref(build: str = "O2"):
    """The compiled reference: oracle/_ref/libref.so (Justfile flags + -O2) or, with
    build="O0", oracle/_ref/libref_O0.so (the Justfile flags as they are: -g, -O0)."""
    path = _REF if build == "O2" else _REF.replace("libref.so", "libref_O0.so")
    if build not in _refs:
        if not os.path.exists(path):
            raise FileNotFoundError(path + " (run `make -C oracle` where /root/reference exists)")
        lib = C.CDLL(path)
        lib.ref_dct_matrix.argtypes = [C.c_int, _dp]
        lib.ref_quant_tables.argtypes = [C.c_int, C.c_int, C.c_int, _dp, _dp, C.POINTER(C.c_int)]
        lib.ref_forward.argtypes = [C.c_int, _dp, _dp]
        lib.ref_inverse.argtypes = [C.c_int, _dp, _dp]
        lib.ref_forward_tables.argtypes = [C.c_int, _dp, _dp, _dp, _dp]
        lib.ref_inverse_tables.argtypes = [C.c_int, _dp, _dp, _dp, _dp]
        lib.ref_variance.argtypes = [C.c_int, _dp]
        lib.ref_variance.restype = C.c_double
        lib.ref_quantize.argtypes = [C.c_int, C.c_int, C.c_int, C.c_double, _dp, _ip]
        lib.ref_dequantize.argtypes = [C.c_int, C.c_int, C.c_int, C.c_double, _ip, _dp]
        lib.ref_adjust.argtypes = [C.c_int, C.c_int, C.c_double, C.c_int, _dp]
        lib.ref_copy_to_coefficients.argtypes = [C.c_int, _dp, _ip]
        lib.ref_forward_plane.argtypes = [_u8p, C.c_int, C.c_int, C.c_int, C.c_int, _i16p, C.c_int, C.c_int]
        lib.ref_rle_encode.argtypes = [C.c_int, _ip, _ip, _ip]
        lib.ref_rle_decode.argtypes = [C.c_int, _ip, _ip, C.c_int, _ip]
        lib.ref_zigzag.argtypes = [C.c_int, _ip, _ip]
        lib.ref_forward_plane.restype = C.c_long
        lib.ref_huffman_bits.argtypes = [C.c_int, _ip, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        lib.ref_huffman_bits.restype = C.c_int
        _refs[build] = lib
    return _refs[build]


# ---------------------------------------------------------------- oracle API
def dct_matrix(n: int = 8) -> np.ndarray:
    d = np.zeros(n * n)
    orc().orc_dct_matrix(n, d)
    return d.reshape(n, n)


def quant_matrix(n: int, quality: int) -> np.ndarray:
    q = np.zeros(n * n)
    orc().orc_quant_matrix(n, quality, q)
    return q.reshape(n, n)


def dequant_matrix(q: np.ndarray) -> np.ndarray:
    n = q.shape[0]
    dq = np.zeros(n * n)
    orc().orc_dequant_matrix(n, np.ascontiguousarray(q, dtype=np.float64).ravel(), dq)
    return dq.reshape(n, n)


def forward(x: np.ndarray) -> np.ndarray:
    n = x.shape[0]
    out = np.zeros(n * n)
    orc().orc_forward(n, dct_matrix(n).ravel(), np.ascontiguousarray(x, np.float64).ravel(), out)
    return out.reshape(n, n)


def inverse(c: np.ndarray) -> np.ndarray:
    n = c.shape[0]
    out = np.zeros(n * n)
    orc().orc_inverse(n, dct_matrix(n).ravel(), np.ascontiguousarray(c, np.float64).ravel(), out)
    return out.reshape(n, n)


def forward_tables(x: np.ndarray, d: np.ndarray, t: np.ndarray) -> np.ndarray:
    """dct_forward on a context whose public tables are d (dct_matrix) and t
    (transposed_dct) as given -- src/dct.c:52-77 reads t in its first pass."""
    n = x.shape[0]
    out = np.zeros(n * n)
    orc().orc_forward_tables(n, np.ascontiguousarray(d, np.float64).ravel(), np.ascontiguousarray(t, np.float64).ravel(),
                             np.ascontiguousarray(x, np.float64).ravel(), out)
    return out.reshape(n, n)


def inverse_tables(c: np.ndarray, d: np.ndarray, t: np.ndarray) -> np.ndarray:
    """dct_inverse with the public tables as given (src/dct.c:80-105)."""
    n = c.shape[0]
    out = np.zeros(n * n)
    orc().orc_inverse_tables(n, np.ascontiguousarray(d, np.float64).ravel(), np.ascontiguousarray(t, np.float64).ravel(),
                             np.ascontiguousarray(c, np.float64).ravel(), out)
    return out.reshape(n, n)


def variance(x: np.ndarray) -> float:
    return orc().orc_variance(x.shape[0], np.ascontiguousarray(x, np.float64).ravel())


def adjust(q: np.ndarray, var: float, is_quantize: int) -> np.ndarray:
    n = q.shape[0]
    m = np.zeros(n * n)
    orc().orc_adjust(n, np.ascontiguousarray(q, np.float64).ravel(), var, is_quantize, m)
    return m.reshape(n, n)


def quantize(c: np.ndarray, quality: int, adaptive: int = 0, var: float = 0.0) -> np.ndarray:
    n = c.shape[0]
    q = np.zeros(n * n, np.int32)
    qm = quant_matrix(n, orc().orc_clamp_quality(quality)).ravel()
    orc().orc_quantize(n, qm, adaptive, var, np.ascontiguousarray(c, np.float64).ravel(), q)
    return q.reshape(n, n)


def dequantize(q: np.ndarray, quality: int, adaptive: int = 0, var: float = 0.0) -> np.ndarray:
    n = q.shape[0]
    c = np.zeros(n * n)
    dq = dequant_matrix(quant_matrix(n, orc().orc_clamp_quality(quality))).ravel()
    orc().orc_dequantize(n, dq, adaptive, var, np.ascontiguousarray(q, np.int32).ravel(), c)
    return c.reshape(n, n)


def forward_plane(px: np.ndarray, quality: int, adaptive: int = 0, nthreads: int = 8,
                  want_float: bool = False):
    """u8 plane [H, W] -> int16 [H/8 * W/8, 64] (and optionally float64 coefficients)."""
    px = np.ascontiguousarray(px, np.uint8)
    h, w = px.shape
    nb = (h // 8) * (w // 8)
    out = np.zeros((nb, 64), np.int16)
    fout = np.zeros((nb, 64), np.float64) if want_float else None
    rc = orc().orc_forward_plane(px.ravel(), w, w, h, quality, adaptive, out.ctypes.data,
                                 fout.ctypes.data if fout is not None else None, nthreads)
    if rc != 0:
        raise ValueError("orc_forward_plane rc=%d" % rc)
    return (out, fout) if want_float else out


def plane_variance(px: np.ndarray) -> np.ndarray:
    px = np.ascontiguousarray(px, np.uint8)
    h, w = px.shape
    var = np.zeros((h // 8) * (w // 8))
    orc().orc_plane_variance(px.ravel(), w, w, h, var)
    return var


def inverse_plane(coef: np.ndarray, quality: int, adaptive: int = 0, var=None) -> np.ndarray:
    coef = np.ascontiguousarray(coef, np.int16).reshape(-1, 64)
    recon = np.zeros(coef.shape, np.float64)
    v = None
    if var is not None:
        var = np.ascontiguousarray(var, np.float64)
        v = var.ctypes.data
    orc().orc_inverse_plane(coef.ravel(), v, coef.shape[0], quality, adaptive, recon.ravel())
    return recon


def synth_plane(seed: int, kind: int, width: int, height: int) -> np.ndarray:
    px = np.zeros((height, width), np.uint8)
    orc().orc_synth_plane(seed, kind, width, height, px.ravel(), width)
    return px


KINDS = {"uniform": 0, "smooth": 1, "const": 2, "extreme": 3}


# ---- zigzag + run-length symbols (src/entropy.c:158-256,327-351) -----------

def zigzag_order(n: int = 8) -> np.ndarray:
    """order[k] = natural (row-major) index of the k-th zigzag element."""
    o = np.zeros(n * n, np.int32)
    orc().orc_zigzag_order(n, o)
    return o


def rle_encode(coeffs: np.ndarray):
    """One block (n x n ints) -> (values, runs) exactly as run_length_encode emits them."""
    c = np.ascontiguousarray(coeffs, np.int32).ravel()
    n = int(round(len(c) ** 0.5))
    v = np.zeros(n * n, np.int32)
    r = np.zeros(n * n, np.int32)
    cnt = orc().orc_rle_encode(n, c, v, r)
    return v[:cnt].copy(), r[:cnt].copy()


def rle_decode(values, runs, n: int = 8) -> np.ndarray:
    v = np.ascontiguousarray(values, np.int32)
    r = np.ascontiguousarray(runs, np.int32)
    out = np.zeros(n * n, np.int32)
    orc().orc_rle_decode(n, v, r, len(v), out)
    return out.reshape(n, n)


def rle_encode_plane(coef: np.ndarray):
    """int16 [nblk, 64] -> (offsets uint32 [nblk+1], symbols uint32 [total]) in the device format:
    symbol = (uint16)value | run << 16, blocks in order."""
    c = np.ascontiguousarray(coef, np.int16).reshape(-1, 64)
    nblk = c.shape[0]
    off = np.zeros(nblk + 1, np.uint32)
    total = orc().orc_rle_encode_plane(c, nblk, off.ctypes.data, None)
    sym = np.zeros(max(total, 1), np.uint32)
    orc().orc_rle_encode_plane(c, nblk, off.ctypes.data, sym.ctypes.data)
    return off, sym[:total]


def pack16(sym: np.ndarray) -> np.ndarray:
    """4-byte symbols ((uint16)value | run << 16) -> the 2-byte format of plans whose
    quantized coefficients all lie in [-511, 511]: (run & 63) << 10 | (value & 0x3FF)
    (uint16).  Runs reach 64 only in the single symbol of an all-zero block, (0, 64)
    (src/entropy.c:231-233: the last element's run counts itself), which becomes 0x0000 --
    a code no other symbol has (a zero value only ends a block, with run >= 1).
    Test infrastructure: a re-encoding of the reference's (value, run) pairs."""
    s = np.ascontiguousarray(sym, np.uint32)
    value = (s & 0xFFFF).astype(np.uint16).view(np.int16).astype(np.int32)
    run = (s >> 16).astype(np.int32)
    if s.size and (np.abs(value).max() > 511 or run.max() > 64 or ((run == 64) & (value != 0)).any()
                   or ((run == 0) & (value == 0)).any()):
        raise ValueError("symbol not representable in 2 bytes")
    return (((run & 63) << 10) | (value & 0x3FF)).astype(np.uint16)


def unpack16(sym16: np.ndarray) -> np.ndarray:
    """The 2-byte format -> 4-byte symbols (pack16's inverse; 0x0000 = (0, 64))."""
    u = np.ascontiguousarray(sym16, np.uint16).astype(np.int32)
    value = ((u & 0x3FF) ^ 0x200) - 0x200
    run = np.where(u == 0, 64, u >> 10)
    return ((value & 0xFFFF) | (run << 16)).astype(np.uint32)


def huffman_bits(coeffs) -> int:
    """One 8x8 int block -> the reference pipeline's per-block size: get_encoded_size after
    build_huffman_codes on its RLE symbols (src/entropy.c:261-328, 363-399)."""
    c = np.ascontiguousarray(coeffs, np.int32).reshape(64)
    return int(orc().orc_huffman_bits(c))


def huffman_bits_plane(coef: np.ndarray) -> np.ndarray:
    """int16 [nblk, 64] -> uint32 [nblk] per-block Huffman sizes (huffman_bits of every block)."""
    c = np.ascontiguousarray(coef, np.int16).reshape(-1, 64)
    out = np.zeros(c.shape[0], np.uint32)
    orc().orc_huffman_bits_plane(c, c.shape[0], out.ctypes.data)
    return out
