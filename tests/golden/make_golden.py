"""Generates tests/golden/*.json from the PYTHON oracle (oracle/py). Run from the repo root:
    python tests/golden/make_golden.py
The reference ships no golden vectors: these fixtures pin our own restatement
(transcript / serialization conventions reconstructed from the unpinned upstream crates, flagged in
oracle/py/transcript.py) so the C oracle and the HIP library can be checked against stored bytes.
Mathematical invariants of the reference are pinned separately in tests/test_oracle_invariants.py."""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle", "py"))

from bls12_381 import G1, G2, R, g1_uncompressed, g2_uncompressed, msm  # noqa: E402
from gen import SplitMix64, ragged, ref_shaped, uniform_3n  # noqa: E402
from spartan import Proof, index, keygen, matrix_bytes, prove, vec_fr_bytes  # noqa: E402
from transcript import Blake2s512Rng, InjectedChallenges  # noqa: E402

CASES = [
    # name, generator, log_n, log_v, seed, param
    ("u3n_4", "uniform_3n", 4, 2, 101, None),
    ("u3n_6", "uniform_3n", 6, 3, 102, None),
    ("ref_5", "ref_shaped", 5, 2, 103, 0),
    ("ref_7_d128", "ref_shaped", 7, 3, 104, 128),
    ("rag_6", "ragged", 6, 2, 105, (3, 1)),
]


def make_instance(gen, log_n, log_v, seed, param):
    if gen == "uniform_3n":
        return uniform_3n(log_n, log_v, seed=seed)
    if gen == "ref_shaped":
        return ref_shaped(log_n, log_v, density=param, seed=seed)
    return ragged(log_n, log_v, param[0], seed, dense_rows=param[1])


def sha(b):
    return hashlib.sha256(b).hexdigest()


def main():
    out = {}
    for name, gen, log_n, log_v, seed, param in CASES:
        A, B, C, v, w = make_instance(gen, log_n, log_v, seed, param)
        n = 1 << log_n
        inst_bytes = matrix_bytes(A, n) + matrix_bytes(B, n) + matrix_bytes(C, n) + vec_fr_bytes(list(v) + list(w))
        pp_seed = 7000 + log_n
        pp, vp, t = keygen(log_n, SplitMix64(pp_seed).next_fr)
        pk = index(A, B, C)
        fs = Blake2s512Rng()
        pf = prove(pk, v, w, pp, fs=fs).to_bytes()
        pfi = prove(pk, v, w, pp, fs=InjectedChallenges(77)).to_bytes()
        # transcript pin: digest right after absorbing A, B, C, v and the first challenges
        tr = Blake2s512Rng()
        for M in (A, B, C):
            tr.feed(matrix_bytes(M, n))
        tr.feed(vec_fr_bytes(v))
        mid = tr.state_digest().hex()
        first = [tr.rand_fr() for _ in range(3)]
        out[name] = {
            "generator": gen,
            "log_n": log_n,
            "log_v": log_v,
            "seed": seed,
            "param": param,
            "pp_seed": pp_seed,
            "instance_sha256": sha(inst_bytes),
            "pp_sha256": sha(pp.serialize_uncompressed()),
            "transcript_digest_after_index_and_v": mid,
            "first_challenges_after_v": [hex(x) for x in first],
            "proof_fs_hex": pf.hex(),
            "proof_injected_seed": 77,
            "proof_injected_hex": pfi.hex(),
        }
        print(name, len(pf), flush=True)
    # MSM known answers (G1 / G2) on keygen bases
    pp, _, _ = keygen(6, SplitMix64(4242).next_fr)
    rs = SplitMix64(99)
    sc = [rs.next_fr() for _ in range(64)]
    sc[3], sc[5], sc[7] = 0, 1, R - 1
    g1b = pp.powers_of_g[0][:64]
    g2b = pp.powers_of_h[0][:48]
    out["msm"] = {
        "pp_seed": 4242,
        "nv": 6,
        "scalars_hex": [x.to_bytes(32, "little").hex() for x in sc],
        "g1_64": g1_uncompressed(G1.to_affine(msm(G1, g1b, sc))).hex(),
        "g2_48": g2_uncompressed(G2.to_affine(msm(G2, g2b, sc[:48]))).hex(),
    }
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
