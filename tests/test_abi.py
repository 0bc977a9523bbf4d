"""CPU: the C-ABI library builds, loads and exports every symbol include/*.h
declares; host-side tables are bit-identical to the reference's; argument
validation fails loudly; no compute is attempted without a GPU."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    from dct_amd.build import build
    build()
    import dct_amd
    return dct_amd.lib()


def declared_functions():
    from dct_amd.build import declared_functions as dec, public_headers
    return set(dec(public_headers()))


def exported(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True).stdout
    return {l.split()[-1] for l in out.splitlines() if " T " in l}


def test_every_declared_symbol_exported(lib):
    names = declared_functions()
    # the reference's per-block API (include/dct.h, quantization.h, utils.h) must all be there
    ref_api = {"dct_init", "dct_free", "dct_forward", "dct_inverse", "create_block_from_pixels",
               "copy_block_to_coefficients", "quant_init", "quant_free", "generate_quant_matrix",
               "generate_dequant_matrix", "quantize", "dequantize", "calculate_block_variance",
               "adjust_matrix_for_block", "alloc_array", "free_array", "alloc_int_array", "free_int_array"}
    assert ref_api <= names, ref_api - names
    # the product library exports exactly what include/*.h declares: no diagnostics, no internals
    got = exported(os.path.join(ROOT, "dct_amd", "libdct_amd.so"))
    assert got == names, (names - got, got - names)
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(ROOT, "dct_amd", "libdct_amd.so")],
                         capture_output=True, text=True).stdout
    assert not [l for l in out.splitlines() if " T " not in l and " A " not in l], "non-function exports"
    for n in names:
        getattr(lib, n)


def test_diagnostic_library_exports(lib):
    """libdct_amd_diag.so = the product's exports + exactly csrc/dctq_diag.h."""
    from dct_amd.build import declared_functions as dec
    diag_names = set(dec([os.path.join(ROOT, "dct_amd", "csrc", "dctq_diag.h")]))
    assert {"dctq_diag_plan_set_variant", "dctq_diag_movement_planes", "dctq_diag_stream",
            "dctq_debug_tables"} <= diag_names
    got = exported(os.path.join(ROOT, "dct_amd", "libdct_amd_diag.so"))
    assert got == declared_functions() | diag_names, got ^ (declared_functions() | diag_names)
    assert not (diag_names & exported(os.path.join(ROOT, "dct_amd", "libdct_amd.so")))


def test_no_runtime_knobs_in_product():
    """Kernel selection is not read from the environment: no getenv in the library sources.
    VERDICT r05 item 6: no compile-time A/B switches in the product sources either (every product
    value is a constexpr; the diagnostic-only DCTQ_ABLATE lives in fdct8_diag.hip), and no
    diagnostic dispatch table behind the product entry points."""
    import re
    csrc = os.path.join(ROOT, "dct_amd", "csrc")
    for f in os.listdir(csrc):
        assert "getenv" not in open(os.path.join(csrc, f)).read(), f
    product = ["fdct8.hip", "roundtrip.hip", "encode.hip", "rle.hip", "huffman.hip", "api.hip", "legacy.hip",
               "f64_pair.hip", "fdct8_aux.hip", "fdct8_core.h", "pair_core.h", "scan_core.h", "dctq_internal.h",
               "plan.h", "aan_f64.h", "zigzag.h", "host_tables.h"]
    for f in product:
        src = open(os.path.join(csrc, f)).read()
        knobs = [m.group(0) for m in re.finditer(r"^#\s*(?:ifndef|ifdef|if|elif)\b.*DCTQ_\w+", src, flags=re.M)
                 if not re.search(r"DCTQ_\w+_H_?\s*$", m.group(0))]
        assert not knobs, (f, knobs)
        assert "g_diag_kernels" not in src and "DiagKernels" not in src, f


def test_host_tables_match_reference(lib, blocks):
    import dct_amd
    for q in [0, 1, 10, 25, 49, 50, 51, 75, 90, 99, 100, 101]:
        w, thr, d, qm = dct_amd.debug_tables(q)
        assert (d.view(np.uint64) == np.array(blocks["dct8"], np.uint64)).all()
        assert (qm.view(np.uint64) == np.array(blocks[f"q8_{q}"], np.uint64)).all(), q
        assert (thr > 0.49).all() and (thr < 0.5).all()
        for adaptive in (0, 1):
            _, thr_a, _, _ = dct_amd.debug_tables(q, adaptive)
            assert (thr_a <= thr + 1e-12).all() if adaptive else True


def test_fastdiv(lib):
    import dct_amd
    lib = dct_amd.diag()
    rng = np.random.default_rng(0)
    for d in [1, 2, 3, 7, 60, 240, 480, 32400, 129600, 8294400, 2**31 - 1]:
        for n in list(rng.integers(0, 2**31 - 1, 200)) + [0, d - 1, d, d + 1, 2**31 - 1]:
            assert lib.dctq_debug_fastdiv(d, int(n)) == int(n) // d, (d, n)


def test_forward_kernel_dispatch(lib):
    """The product forward (fdct8.hip): in-place ties (v3) for every plan at every size.
    Since round 4 that includes tie-heavy plans (q >= 97: DC divisor 1, the rational
    coefficients tie in ~1 block of 8), which ran on the queue kernel (v2) before
    (profiles/r04/v3_tieheavy_ab.log); since round 5 v2 is not in the product at all."""
    import dct_amd
    big, small = 194400, 4096  # the bench step's batches; 16 waves per CU x 256 CUs
    for q in (1, 10, 50, 90, 95, 96):
        for ad in (0, 1):
            assert dct_amd.forward_kernel(q, ad, big, 256).startswith("fdct8_quant_v3"), (q, ad)
    for q in (97, 99, 100):
        assert dct_amd.debug_tables(q)[3][0] <= 1.0
        assert dct_amd.forward_kernel(q, 0, big, 256).startswith("fdct8_quant_v3"), q
        assert dct_amd.forward_kernel(q, 0, small, 256).startswith("fdct8_quant_v3"), q
    assert dct_amd.forward_kernel(50, 1, big, 256) == "fdct8_quant_v3<true, false, false>"


def _device_kernels(path, tmp):
    """Kernel symbols of every gfx950 code object embedded in a library
    (llvm-objdump --offloading extracts them, llvm-readelf lists their symbols)."""
    import glob
    import shutil
    llvm = "/opt/rocm/lib/llvm/bin"
    os.makedirs(tmp, exist_ok=True)
    local = os.path.join(tmp, os.path.basename(path))
    shutil.copy(path, local)
    r = subprocess.run([os.path.join(llvm, "llvm-objdump"), "--offloading", local], cwd=tmp, capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stderr
    names = set()
    objs = glob.glob(local + ".*gfx950")
    assert objs, os.listdir(tmp)
    for obj in objs:
        out = subprocess.run([os.path.join(llvm, "llvm-readelf"), "--symbols", obj], capture_output=True,
                             text=True).stdout
        names |= {w for w in out.split() if w.startswith("_Z") and "." not in w}
    return names


def test_product_code_object_has_only_product_kernels(lib, tmp_path):
    """the retired forward kernels (v1, the v2 tie queue), the
    lane-per-block fp64 variants and the no-arithmetic movement twins are built into
    libdct_amd_diag.so only (csrc/fdct8_diag.hip); the product's code objects hold the
    kernels the product dispatch runs."""
    prod = _device_kernels(os.path.join(ROOT, "dct_amd", "libdct_amd.so"), str(tmp_path / "p"))
    diag = _device_kernels(os.path.join(ROOT, "dct_amd", "libdct_amd_diag.so"), str(tmp_path / "d"))
    retired = ("fdct8_quant_v1", "fdct8_quant_v2", "fdct8_movement", "roundtrip_movement", "fdct8_float_kernel",
               "idct8_kernel")
    assert not [k for k in prod if any(r in k for r in retired)], sorted(prod)
    for want in ("fdct8_quant_v3", "roundtrip8ILb0ELb0ELb0ELb1", "roundtrip8ILb1ELb0ELb0ELb0", "idct8_pair", "fdct8_float_pair",
                 "encode_count_kernel", "huffman_bits_kernel", "synth_kernel"):
        assert any(want in k for k in prod), (want, sorted(prod))
    for r in retired:
        assert any(r in k for k in diag), (r, sorted(diag))


def test_error_strings(lib):
    import dct_amd
    assert dct_amd.lib().dctq_error_string(0) == b"ok"
    assert dct_amd.lib().dctq_error_string(-1)


def test_c_hosts_compile_and_link(lib):
    out = subprocess.run(["make", "-C", os.path.join(ROOT, "host")], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr


def test_headers_compile_as_c99(tmp_path):
    src = tmp_path / "t.c"
    src.write_text('#include "dct.h"\n#include "quantization.h"\n#include "utils.h"\n#include "dct_amd.h"\n'
                   "int main(void){DCTContext c; QuantContext q; dctq_plane p; (void)c; (void)q; (void)p; return 0;}\n")
    out = subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-pedantic",
                          "-I" + os.path.join(ROOT, "include"), "-c", str(src), "-o", str(tmp_path / "t.o")],
                         capture_output=True, text=True)
    assert out.returncode == 0, out.stderr


def test_struct_layouts_match_reference():
    """DCTContext / QuantContext are public in the reference (include/dct.h:21-25,
    include/quantization.h:18-24): same field order, offsets and size."""
    code = r'''
#include <stddef.h>
#include <stdio.h>
#include "dct.h"
#include "quantization.h"
int main(void){
 printf("%zu %zu %zu %zu\n", sizeof(DCTContext), offsetof(DCTContext, block_size), offsetof(DCTContext, dct_matrix), offsetof(DCTContext, transposed_dct));
 printf("%zu %zu %zu %zu %zu %zu\n", sizeof(QuantContext), offsetof(QuantContext, block_size), offsetof(QuantContext, quality), offsetof(QuantContext, quant_matrix), offsetof(QuantContext, dequant_matrix), offsetof(QuantContext, adaptive));
 return 0;}
'''
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        res = {}
        incs = {"ours": os.path.join(ROOT, "include")}
        if os.path.isdir("/root/reference/include"):
            incs["ref"] = "/root/reference/include"
        for tag, inc in incs.items():
            p = os.path.join(td, f"{tag}.c")
            open(p, "w").write(code)
            exe = os.path.join(td, tag)
            out = subprocess.run(["gcc", "-std=c99", "-I" + inc, p, "-o", exe], capture_output=True, text=True)
            assert out.returncode == 0, out.stderr
            res[tag] = subprocess.run([exe], capture_output=True, text=True).stdout
        assert res["ours"].split() == ["24", "0", "8", "16", "32", "0", "4", "8", "16", "24"]
        if "ref" in res:
            assert res["ours"] == res["ref"]


def test_constant_block_dc_table(lib):
    """The per-plan table of quantized DCs of constant blocks (flat-block tie
    resolution in the forward kernel) equals the oracle's reference-order
    forward + quantize of each constant block."""
    import oracle as O
    import dct_amd
    lib = dct_amd.diag()
    for q in [1, 10, 25, 50, 75, 90, 100]:
        tab = np.zeros(256, np.int16)
        assert lib.dctq_debug_dc_table(q, tab.ctypes.data) == 0
        for v in range(256):
            x = np.full((8, 8), v - 128.0)
            want = O.quantize(O.forward(x), q, 0, 0.0)[0, 0]
            assert tab[v] == want, (q, v, tab[v], want)
            assert O.quantize(O.forward(x), q, 1, O.variance(x))[0, 0] == want  # adaptive keeps Q for the DC


def test_build_manifest_matches_library():
    """build() is content-gated: dct_amd/build_info.json records the sha256 of every
    source, header and flag the libraries were built from and of the two libraries;
    the shipped libdct_amd.so is the one it describes (bench.py reports the same
    hash in its `build` record)."""
    import hashlib

    from dct_amd import build as B
    info = B.build_info()
    assert info, "dct_amd/build_info.json missing: run python -m dct_amd.build"
    assert info["lib_sha256"] == hashlib.sha256(open(B.LIB, "rb").read()).hexdigest()
    assert info["diag_sha256"] == hashlib.sha256(open(B.DIAG_LIB, "rb").read()).hexdigest()
    assert info["inputs"] == B._inputs(), "sources changed since the last build"
    assert not B._stale()
