"""The batch descriptor tag (csrc/pf_desc_tag.hpp), on the CPU.

pfmpe_step_multi tags every stream descriptor; the staging kernel recomputes the tag over the words it read
and refuses a descriptor whose tag or generation differs (tests/test_gpu_multi.py corrupts one on purpose).
Here the same header is built with g++: a single changed word must always change the tag (tag_mix is a
bijection per position), random multi-word changes must change it, and the value must equal an independent
Python restatement of the function.
"""
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
M64 = (1 << 64) - 1


def tag_mix(w, i):
    z = (w + 0x9E3779B97F4A7C15 * (i + 1)) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def desc_tag(words):
    h = 0
    for i, w in enumerate(words):
        h ^= tag_mix(w, i)
    return h


def test_desc_tag_detects_changes_and_matches_restatement(tmp_path):
    exe = tmp_path / "desc_tag_check"
    subprocess.run(["g++", "-std=c++11", "-O2", "-Wall", "-Wextra", os.path.join(ROOT, "tests", "desc_tag_check.cpp"),
                    "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.split()
    words = [((0x0123456789abcdef * (i + 1)) & M64) ^ (i << 7) for i in range(130)]
    assert int(lines[0], 16) == desc_tag(words)
    assert lines[1] == "ok"


def test_tag_mix_is_a_bijection_sample():
    rng = np.random.default_rng(3)
    ws = [int(x) for x in rng.integers(0, 2 ** 63, size=2000, dtype=np.int64)]
    for i in (0, 1, 77):
        assert len({tag_mix(w, i) for w in ws}) == len(set(ws))
