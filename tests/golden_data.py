"""Loaders for the committed golden fixtures (tests/golden/, made by make_golden.py)."""
from __future__ import annotations

import json
import os

import numpy as np

from picotcp_amd import synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DESC_DTYPE = np.dtype([("off", "<u8"), ("len", "<u4"), ("seed", "<u4")])


def kat() -> dict:
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        return json.load(f)


def raw_cases() -> dict:
    z = np.load(os.path.join(GOLDEN, "raw_cases.npz"))
    cases: dict = {}
    for key in z.files:
        name, field = key.split("__")
        cases.setdefault(name, {})[field] = z[key]
    return cases


def raw_case_inputs(case: dict, seed_fn):
    """(buffer, desc) for a raw case; seed_fn(first12_bytes) -> accumulator seed."""
    buf = synth.random_bytes(int(case["buf_seed"]), int(case["buf_len"]))
    n = case["off"].size
    first = synth.random_bytes(int(case["buf_seed"]) ^ 0x77, 12 * n).reshape(n, 12)
    desc = np.zeros(n, dtype=DESC_DTYPE)
    desc["off"] = case["off"]
    desc["len"] = case["len"]
    for i in np.nonzero(case["first_len"])[0]:
        desc["seed"][i] = seed_fn(first[i, :case["first_len"][i]])
    return buf, desc


def ipv4_cases() -> dict:
    z = np.load(os.path.join(GOLDEN, "ipv4_cases.npz"))
    return {k: z[k] for k in z.files}


def unit_socket_frames() -> dict:
    z = np.load(os.path.join(GOLDEN, "unit_socket_frames.npz"))
    return {k: z[k] for k in z.files}


def ipv4_desc(net: np.ndarray, avail: np.ndarray) -> np.ndarray:
    d = np.zeros(net.size, dtype=DESC_DTYPE)
    d["off"] = net
    d["len"] = avail
    return d


def ipv6_cases() -> dict:
    z = np.load(os.path.join(GOLDEN, "ipv6_cases.npz"))
    return {k: z[k] for k in z.files}


def ipv6_desc(c: dict) -> np.ndarray:
    d = ipv4_desc(c["net"], c["avail"])
    d["seed"] = c["seed"]
    return d


def ref_callers() -> dict:
    """Transport checksums from the reference's own compiled callers (make_ref_callers.py)."""
    z = np.load(os.path.join(GOLDEN, "ref_callers.npz"))
    return {k: z[k] for k in z.files}


def eth_cases() -> dict:
    """Mixed Ethernet burst with the oracle_batch_eth expectations (make_ref_callers.py)."""
    z = np.load(os.path.join(GOLDEN, "eth_cases.npz"))
    return {k: z[k] for k in z.files}


def eth_desc(c: dict, rx: bool = True) -> np.ndarray:
    d = np.zeros(c["off"].size, dtype=DESC_DTYPE)
    d["off"] = c["off"]
    d["len"] = c["rx_len"] if rx else c["flen"]
    d["seed"] = c["seed"]
    return d


def ref_rx_cases() -> dict:
    """Datagrams with the reference's own RX verdicts (make_ref_rx.py)."""
    z = np.load(os.path.join(GOLDEN, "ref_rx_cases.npz"))
    return {k: z[k] for k in z.files}


def ref_reasm_cases() -> dict:
    """Fragment groups with the reference's own reassembly results (make_ref_reasm.py)."""
    z = np.load(os.path.join(GOLDEN, "ref_reasm_cases.npz"))
    return {k: z[k] for k in z.files}


def ref_eth_cases() -> dict:
    """An Ethernet burst with the reference's own L2 + IP verdicts (make_ref_eth.py)."""
    z = np.load(os.path.join(GOLDEN, "ref_eth_cases.npz"))
    return {k: z[k] for k in z.files}
