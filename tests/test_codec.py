"""Frontier record codec (rmc_spec.h Codec) round trip, compiled for the host with g++.

The kernels compute on the nibble layout and store the packed form in HBM; a field that does
not survive encode -> decode would silently change states, so every compiled (servers, values)
instantiation is checked on random states drawn from the spec's field domains."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_codec_round_trip(tmp_path):
    exe = tmp_path / "codec_rt"
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "tla-raft_amd", "csrc"),
                           os.path.join(ROOT, "tests", "codec_roundtrip.cpp"), "-o", str(exe)])
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "N=3 V=2: 128 bits in 4 words, 0 mismatches" in r.stdout
