"""The kernels' host-emulated item functions under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5
host sanitizer tests): tests/emu/emu_asan_main.cpp includes the emulator (tests/emu/emu.cpp, the same
fft_core.h / slab_ct.h / kspace_ct.h / sap_core.h the gfx950 kernels compile) into one executable built with
-fsanitize=address,undefined, and runs the full-spectrum passes on odd / even / prime / padded shapes, a
compiled slab plan, the Philox stream, the salt-and-pepper classes and the min/max keys.  A sanitizer finding
aborts the run; an invariant violation exits non-zero.  CPU only."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(ROOT, "medical-vision-textural-bias_amd", "csrc")
SRC = [os.path.join(HERE, "emu", "emu_asan_main.cpp"), os.path.join(HERE, "emu", "emu.cpp")] + \
      [os.path.join(CSRC, h) for h in ("fft_core.h", "slab_ct.h", "kspace_ct.h", "plan_host.h", "sap_core.h")]
EXE = os.path.join(HERE, "emu", "_build", "emu_asan")


def test_emulator_under_asan_ubsan():
    newest = max(os.path.getmtime(p) for p in SRC)
    if not os.path.exists(EXE) or os.path.getmtime(EXE) < newest:
        os.makedirs(os.path.dirname(EXE), exist_ok=True)
        tmp = EXE + f".{os.getpid()}.tmp"
        cxx = os.environ.get("TB_EMU_CXX", "/opt/rocm/lib/llvm/bin/clang++")
        subprocess.check_call([cxx, "-O0", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                               "-Wno-unknown-pragmas", "-I", os.path.join(ROOT, "include"), "-I", CSRC, SRC[0], "-o", tmp])
        os.replace(tmp, EXE)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "emu sanitizer run ok" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
