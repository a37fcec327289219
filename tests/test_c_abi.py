"""The C host boundary from plain C: tests/c_abi/abi_check.c (gcc, include/pico_csum.h,
libpicocsum.so; no Python in the loop) runs the fused IPv4 device batch, the
host-resident uniform batch and the scalar drop-in against tests/golden/c_abi_burst.bin
(made by tests/golden/make_c_abi_golden.py from the oracle)."""
from __future__ import annotations

import os
import subprocess

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
EXE = os.path.join(ROOT, "tests", "c_abi", "abi_check")
FIX = os.path.join(ROOT, "tests", "golden", "c_abi_burst.bin")


def _exe():
    if not os.path.exists(EXE):
        pytest.fail(f"{EXE} not built: run __graft_entry__.build() (make -C tests/c_abi)")
    return EXE


def test_c_abi_check_refuses_without_device():
    """CPU container: the program loads the library, reads the fixture and reports the
    missing device with its own exit status (2), never a silent pass."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present")
    r = subprocess.run([_exe(), FIX], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2, r.stderr


@pytest.mark.gpu
def test_c_abi_check_on_gpu():
    r = subprocess.run([_exe(), FIX], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok" in r.stdout
