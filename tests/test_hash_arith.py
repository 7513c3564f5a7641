"""The MinMax query's integer shortcuts (skml_sparse.hip: k / 1000 as a double product, BKDR
chunks with 24-bit multiplies, the 32-bit floor modulus) against the reference's own arithmetic
(hash/BKDRHash.java:13-21, Int2IntHash's `code % size`), checked on the host: every 32-bit k for
k / 1000, every key below 2^24 and 4 M random keys per BKDR seed, and modulus edges."""
import os
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_hash_shortcuts_match_reference_arithmetic():
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "hash_arith_check")
        subprocess.run(["gcc", "-O2", "-std=c11", "-o", exe, os.path.join(ROOT, "tests", "hash_arith_check.c"), "-lm"],
                       check=True)
        out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stdout
