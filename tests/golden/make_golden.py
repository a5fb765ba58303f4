"""Regenerate tests/golden/derived_vectors.json from the CPU oracle.

The oracle is first pinned by reference_vectors.json (the reference's own
known answers); these derived fixtures extend that pin to the geometries the
benchmark uses (matrix rows, and digests of encoded synthetic stripes) so the
GPU tests can check full-size outputs without re-running the oracle.
Run: python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402


def main():
    out = {"_about": "Derived from the oracle pinned by reference_vectors.json; regenerate with make_golden.py",
           "parity_rows": {}, "stripes": []}
    for k, m in [(2, 2), (4, 2), (6, 3), (8, 4), (12, 4), (16, 4)]:
        out["parity_rows"][f"{k},{m}"] = [bytes(r).hex() for r in O.matrix(k, m)[k:]]
    rng = np.random.default_rng(20260821)
    for k, m, S in [(2, 2, 4096), (4, 2, 1890), (8, 4, 8192), (8, 4, 1000), (16, 4, 4096), (6, 2, 3001)]:
        data = rng.integers(0, 256, (k, S), dtype=np.uint8)
        st = np.zeros((k + m, S), dtype=np.uint8)
        st[:k] = data
        O.encode(k, m, st)
        out["stripes"].append({
            "k": k, "m": m, "S": S, "seed": 20260821,
            "data_sha256": hashlib.sha256(data.tobytes()).hexdigest(),
            "parity_sha256": hashlib.sha256(st[k:].tobytes()).hexdigest(),
            "hh256s": [O.hh256s(st[i]).hex() for i in range(k + m)],
        })
    with open(os.path.join(ROOT, "tests", "golden", "derived_vectors.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
