"""CPU: the repository's CPU-side C under AddressSanitizer + UndefinedBehaviorSanitizer
(VERDICT r01 item 8).

* tests/san/san_check.c drives the oracle (oracle/dct_oracle.c, incl. its
  pthread plane loops) and, where /root/reference exists, the reference's own
  src/*.c through oracle/ref_driver.c, bit for bit against each other, all
  compiled with -fsanitize=address,undefined -fno-sanitize-recover=all;
* the C hosts (host/*.c) are compiled and linked with the same flags against
  libdct_amd.so (running them needs a GPU);
* the host side of the library (every .hip source, device code untouched) is
  compiled with -Xarch_host -fsanitize=address,undefined, so the HIP build
  accepts the instrumented host objects.
A finding aborts the program, so a clean exit is the pass condition."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]


def run(cmd, **kw):
    out = subprocess.run(cmd, capture_output=True, text=True, **kw)
    assert out.returncode == 0, " ".join(cmd) + "\n" + out.stdout[-4000:] + out.stderr[-4000:]
    return out


def test_oracle_and_reference_under_asan_ubsan(tmp_path):
    srcs = [os.path.join(ROOT, "tests", "san", "san_check.c"), os.path.join(ROOT, "oracle", "dct_oracle.c")]
    flags = ["-std=c99", "-Wall", "-Wextra", "-Werror", "-ffp-contract=off", "-I" + os.path.join(ROOT, "oracle")]
    if os.path.exists(os.path.join(REF, "src", "dct.c")):
        flags.append("-I" + os.path.join(REF, "include"))
        srcs += [os.path.join(ROOT, "oracle", "ref_driver.c")] + [os.path.join(REF, "src", f) for f in
                                                                  ("utils.c", "dct.c", "quantization.c", "entropy.c")]
    else:
        flags.append("-DNO_REF")
    exe = str(tmp_path / "san_check")
    # -pedantic off: the reference's sources are compiled as they are
    run(["gcc", *flags, *SAN, *srcs, "-o", exe, "-lm", "-lpthread"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    out = run([exe], env=env, timeout=600)
    assert "0 failure(s)" in out.stdout


def test_c_hosts_build_with_sanitizers(tmp_path):
    from dct_amd.build import build
    build()
    for src in sorted(os.listdir(os.path.join(ROOT, "host"))):
        if src.endswith(".c"):
            run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-pedantic", *SAN, "-I" + os.path.join(ROOT, "include"),
                 os.path.join(ROOT, "host", src), "-L" + os.path.join(ROOT, "dct_amd"), "-ldct_amd", "-lm",
                 "-o", str(tmp_path / src[:-2])])


@pytest.mark.parametrize("src", ["api.hip", "legacy.hip", "diag.hip"])
def test_library_host_code_builds_with_sanitizers(src, tmp_path):
    csrc = os.path.join(ROOT, "dct_amd", "csrc")
    run(["hipcc", "--offload-arch=gfx950", "-O1", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
         "-I" + os.path.join(ROOT, "include"), "-I" + csrc, "-c", os.path.join(csrc, src),
         "-o", str(tmp_path / (src + ".o"))])
