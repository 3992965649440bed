"""Sanitizer builds of the host-side code: the CPU oracle and the product's host library
(libspg_hostcheck: field / curve / transcript / round-polynomial / cross-rank exchange code that the HIP
sources share) under AddressSanitizer + UndefinedBehaviorSanitizer, and the host worker pool plus the
cross-rank exchange under ThreadSanitizer. The ASan run re-executes the oracle and product-host test modules
in a subprocess with libasan preloaded (Python itself is not instrumented); any report fails the run."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "spartan-parallel_amd")


def _rt(name):
    return subprocess.check_output(["gcc", f"-print-file-name={name}"], text=True).strip()


def test_pool_and_exchange_under_tsan():
    subprocess.check_call(["make", "-s", "-C", PKG, "lib/spg_pool_tsan"])
    out = subprocess.run([os.path.join(PKG, "lib", "spg_pool_tsan")], capture_output=True, text=True, timeout=300,
                         env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1"))
    assert out.returncode == 0, out.stdout + out.stderr[-4000:]
    assert "ThreadSanitizer" not in out.stderr, out.stderr[-4000:]
    assert "0 violations" in out.stdout


def test_oracle_and_product_host_under_asan_ubsan():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"])
    subprocess.check_call(["make", "-s", "-C", PKG, "lib/libspg_hostcheck_asan.so"])
    env = dict(os.environ,
               LD_PRELOAD=_rt("libasan.so"),
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               ORACLE_LIB=os.path.join(ROOT, "oracle", "build", "liboracle_asan.so"),
               SPG_HOSTCHECK_LIB=os.path.join(PKG, "lib", "libspg_hostcheck_asan.so"))
    mods = ["tests/test_oracle_core.py", "tests/test_product_host.py", "tests/test_oracle_r1cs.py",
            "tests/test_oracle_spark.py"]
    out = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", *mods], cwd=ROOT,
                         env=env, capture_output=True, text=True, timeout=900)
    tail = out.stdout[-3000:] + out.stderr[-3000:]
    assert out.returncode == 0, tail
    assert "AddressSanitizer" not in out.stderr and "runtime error" not in out.stderr, tail
