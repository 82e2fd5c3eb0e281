"""Generate the golden fixtures under tests/golden/ (run from the repo root:
``python tests/golden/make_golden.py``).

Provenance of every fixture:
* kat_stability.json — copied DATA from the reference's own known-answer table,
  repo/splitter/splitter_test.go:27-52 (count, avg, min, max over 5,000,000 bytes
  of rand.NewSource(5)); plus the MaxSegmentSize pins.
* check_values.json — Go math/rand / rollinghash check values listed in
  SURVEY.md Appendix A (public Go stdlib constants and module outputs) and the
  object-writer FIXED pins (repo/object/object_manager_test.go:216-264).
* tables.json, cuts_*.json — outputs of the oracle (oracle/), which is pinned by
  the two files above (tests/test_oracle.py re-checks that).

The reference is Go and cannot run here (no Go toolchain), so no
fixture is produced by executing the reference itself.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import coracle, gorand, rollinghash  # noqa: E402
from oracle.splitter_ref import REGISTRY, supported_algorithms  # noqa: E402

KAT = [  # repo/splitter/splitter_test.go:27-52  (factory, count, avg, minSplit, maxSplit)
    ["fixed", 1000, 5000, 1000, 1000, 1000, False],
    ["fixed", 10000, 500, 10000, 10000, 10000, False],
    ["buzhash", 32, 124235, 40, 16, 64, False],
    ["buzhash", 1024, 3835, 1303, 512, 2048, False],
    ["buzhash", 2048, 1924, 2598, 1024, 4096, False],
    ["buzhash", 32768, 112, 44642, 16413, 65536, False],
    ["buzhash", 65536, 57, 87719, 32932, 131072, False],
    ["rabinkarp", 32, 124108, 40, 16, 64, False],
    ["rabinkarp", 1024, 3771, 1325, 512, 2048, False],
    ["rabinkarp", 2048, 1887, 2649, 1028, 4096, False],
    ["rabinkarp", 32768, 121, 41322, 16896, 65536, False],
    ["rabinkarp", 65536, 53, 94339, 35875, 131072, False],
    ["fixed", 1000, 5000, 1000, 1000, 1000, True],
    ["buzhash", 32, 124235, 40, 16, 64, True],
    ["buzhash", 1024, 3835, 1303, 512, 2048, True],
    ["buzhash", 2048, 1924, 2598, 1024, 4096, True],
    ["buzhash", 32768, 112, 44642, 16413, 65536, True],
    ["buzhash", 65536, 57, 87719, 32932, 131072, True],
    ["rabinkarp", 32, 124108, 40, 16, 64, True],
    ["rabinkarp", 1024, 3771, 1325, 512, 2048, True],
    ["rabinkarp", 2048, 1887, 2649, 1028, 4096, True],
    ["rabinkarp", 32768, 121, 41322, 16896, 65536, True],
    ["rabinkarp", 65536, 53, 94339, 35875, 131072, True],
]

CHECK = {
    "rng_cooked_first3": [-4181792142133755926, -4576982950128230565, 1395769623340756751],
    "rng_cooked_606": 4152330101494654406,
    "rng_cooked_sha256": "1928503b93a563e491119a5889baba73d1605b90b63634c14a408805797a7c7b",
    "seed1_int63": [5577006791947779410, 8674665223082153551, 6129484611666145821, 4037200794235010051],
    "seed5_read5e6_sha256": "d420cd9782f8d6444e15f6678036cf2677dab335327ab73a98d38fb19d2cfd6f",
    "seed42_read1MiB_sha256": "b53d2e2c84e19771c5a80f27ac78ff4d48f12972ff87f6ef07962b6ffb832656",
    "buzhash_first4": ["07fcfd52", "5f3f164f", "6695721d", "7b4d7c03"],
    "buzhash_255": "4cf20a65",
    "buzhash_sha256": "8b089027ee3aa8dc8ed3311bae87113e09c4aaefb631b701f670a9d99c4c3e63",
    "rabin_pol": "0x2e3e3e4a305605",
    "rabin_tries": 106,
    "rabin_out1": "0x18c8237bf89981",
    # repo/object/object_manager_test.go:216-264: 128<<10 copies of an 11-byte pattern
    "fixed_object_lengths": {"FIXED-1M": [1048576, 393216], "FIXED-128K": [131072] * 11,
                             "FIXED-256K": [262144] * 5 + [131072]},
}

EDGE_NAMES = ["DYNAMIC-128K-BUZHASH", "DYNAMIC-128K-RABINKARP"]


def edge_inputs():
    """Deterministic edge-case streams (regenerable on the GPU box without the
    reference): lengths around min/max of the 128K variants, all-zero data and
    the 11-byte periodic pattern."""
    K = 128 << 10
    mn, mx = K // 2, 2 * K
    out = {}
    for L in [0, 1, 63, 64, 65, mn - 1, mn, mn + 1, mx - 1, mx, mx + 1, 3 * mx + 17]:
        out[f"prng_len_{L}"] = ("prng", L)
    out["zeros_5x"] = ("zeros", 5 * mx + 3)
    out["pattern11"] = ("pattern11", 11 * (128 << 10))
    return out


def materialize(kind: str, n: int) -> np.ndarray:
    if kind == "prng":
        return coracle.gen_stream(0x6B6F706961, 7, n)
    if kind == "zeros":
        return np.zeros(n, dtype=np.uint8)
    if kind == "pattern11":
        return np.tile(np.arange(1, 12, dtype=np.uint8), n // 11 + 1)[:n]
    raise ValueError(kind)


def main():
    # tables
    out, mod = rollinghash.rabin_tables()
    P, tries = rollinghash.rabin_polynomial()
    tables = {
        "buzhash": [f"{int(x):08x}" for x in rollinghash.buzhash_table()],
        "rabin_pol": hex(P), "rabin_tries": tries,
        "rabin_out": [f"{int(x):016x}" for x in out],
        "rabin_mod": [f"{int(x):016x}" for x in mod],
        "rng_cooked_sha256": gorand.rng_cooked_sha256(),
    }
    json.dump(tables, open(os.path.join(HERE, "tables.json"), "w"), indent=0)
    json.dump({"kat": KAT, "data": {"seed": 5, "len": 5000000}}, open(os.path.join(HERE, "kat_stability.json"), "w"),
              indent=1)
    json.dump(CHECK, open(os.path.join(HERE, "check_values.json"), "w"), indent=1)

    # full cut lists of the reference KAT input for every registered name (oracle output)
    data = coracle.gorand_read(5, 5_000_000)
    assert hashlib.sha256(data.tobytes()).hexdigest() == CHECK["seed5_read5e6_sha256"]
    cuts = {name: coracle.split_stream(name, data).tolist() for name in supported_algorithms()}
    json.dump({"input": "rand.NewSource(5).Read(5000000)", "cuts": cuts},
              open(os.path.join(HERE, "cuts_kat_input.json"), "w"))

    # edge inputs
    edge = {}
    for key, (kind, n) in edge_inputs().items():
        d = materialize(kind, n)
        edge[key] = {"kind": kind, "len": n,
                     "cuts": {nm: coracle.split_stream(nm, d).tolist() for nm in EDGE_NAMES + ["FIXED-128K"]}}
    json.dump({"prng_seed": 0x6B6F706961, "prng_sid": 7, "cases": edge},
              open(os.path.join(HERE, "cuts_edge.json"), "w"))
    print("wrote", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    main()
