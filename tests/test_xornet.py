"""The generated RS(8,4) XOR network (rustfs_amd/csrc/rs84_xornet.h, used by
the fused encode+HH256S kernel's encoder waves) checked on the CPU: the
header's straight-line program is parsed and evaluated on bit planes of
random data, and the parity bytes it yields must equal the oracle's RS(8,4)
encode (the reference's Vandermonde construction, erasure.rs:448-470).  The
GPU parity tests check the kernel itself; this pins the generated network
independently of any device."""
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "rustfs_amd", "csrc", "rs84_xornet.h")


def _program():
    body = open(HEADER).read()
    body = body[body.index("rs84_encode_planes"):]
    stmts = re.findall(r"(?:const uint32_t (t\d+)|O\[(\d+)\]) = (.+?);", body)
    assert stmts, "no statements parsed"
    return stmts


def _eval(expr: str, env: dict) -> int:
    # the expressions use only x3(a, b, c), a ^ b, P[i], tN and 0u
    py = expr.replace("0u", "0")
    py = re.sub(r"P\[(\d+)\]", r"P[\1]", py)
    return eval(py, {"x3": lambda a, b, c: a ^ b ^ c}, env)


def _planes(data: np.ndarray) -> list:
    """data (8, 32) bytes -> 64 planes: plane c*8+j bit q = bit j of data[c][q]."""
    P = []
    for c in range(8):
        for j in range(8):
            bits = (data[c] >> j) & 1
            P.append(int(sum(int(b) << q for q, b in enumerate(bits))))
    return P


def test_xornet_matches_oracle_encode(oracle):
    stmts = _program()
    n_ops = sum(1 for t, o, e in stmts if t or "x3" in e or "^" in e)
    assert n_ops < 504, "the network must beat folding each output plane separately"
    rng = np.random.default_rng(84)
    for trial in range(16):
        data = rng.integers(0, 256, (8, 32), dtype=np.uint8)
        if trial == 0:
            data[:] = 0
        elif trial == 1:
            data[:] = 0xFF
        env = {"P": _planes(data)}
        O = [None] * 32
        for t, o, expr in stmts:
            v = _eval(expr, env)
            if t:
                env[t] = v
            else:
                O[int(o)] = v
        got = np.zeros((4, 32), dtype=np.uint8)
        for r in range(4):
            for i in range(8):
                for q in range(32):
                    got[r, q] |= ((O[8 * r + i] >> q) & 1) << i
        st = np.zeros((12, 32), dtype=np.uint8)
        st[:8] = data
        oracle.encode(8, 4, st)
        assert np.array_equal(got, st[8:]), trial
