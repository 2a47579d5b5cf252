"""The host weight packers (tts-3_amd/csrc/pack.cpp) under AddressSanitizer + UBSan:
`make -C tts-3_amd asan-check` builds csrc/pack.cpp with tests_native/pack_check.cpp, packs every
layout (conv1d fp32 fragments, the three split modes, ConvTranspose both ways, Winograd) into
buffers of exactly packed_*_numel elements, decodes them back against the torch weights and
checks the non-finite-weight error path."""
import os
import shutil
import subprocess

import pytest

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tts-3_amd")


@pytest.mark.skipif(shutil.which("make") is None or not os.path.exists("/opt/rocm/llvm/bin/clang++"),
                    reason="needs make and the ROCm clang++")
def test_packers_clean_under_asan_ubsan():
    r = subprocess.run(["make", "-C", PKG, "asan-check"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "all packers OK" in r.stdout
