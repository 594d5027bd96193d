"""ORACLE — TEST INFRASTRUCTURE ONLY.

Fiat–Shamir transcript of the reference: `linear_sumcheck::data_structures::Blake2s512Rng`
[upstream arkworks-rs/sumcheck, unpinned git dep, Cargo.toml:15; not in container],
driven from /root/reference/src/lib.rs:61-131 and the `sample_*` functions of
/root/reference/src/ahp/verifier.rs:172-178,211-217,269-273,301-307,354-360,434-440.

Reconstructed semantics ("unverified against upstream"):
  * state = Blake2s (32-byte digest, the `blake2` crate's `Blake2s::default()`);
  * `feed_randomness(m)` = update(state, ark-serialize(m) compressed bytes);
  * `fill_bytes(dest)`: out = finalize(clone(state)); copy bytes of `out` into dest; whenever
    all 32 bytes of `out` are consumed: update(state, out), out = finalize(clone(state));
    after dest is full: update(state, out);
  * `next_u64` = fill_bytes(8) little-endian;
  * `Fr::rand` (ark-ff UniformRand for Fp256): 4 x next_u64 -> BigInteger256 limbs, mask the
    top limb with u64::MAX >> REPR_SHAVE_BITS (=1), retry while >= r; the accepted bigint is the
    Montgomery REPRESENTATION, so the field value is v * R^-1 mod r.

`InjectedChallenges` is the "mode=injected" source: it ignores feeds and
returns a fixed SplitMix64 stream, isolating transcript-convention risk from kernel parity.
"""
import hashlib

from bls12_381 import R, fr_from_mont_limbs
from gen import SplitMix64


class Blake2s512Rng:
    def __init__(self):
        self.h = hashlib.blake2s()

    def feed(self, data: bytes):
        self.h.update(data)

    def fill_bytes(self, n):
        out = bytearray()
        output = self.h.copy().digest()
        ptr = 0
        while len(out) < n:
            out.append(output[ptr])
            ptr += 1
            if ptr == len(output):
                self.h.update(output)
                output = self.h.copy().digest()
                ptr = 0
        self.h.update(output)
        return bytes(out)

    def next_u64(self):
        return int.from_bytes(self.fill_bytes(8), "little")

    def rand_fr(self):
        while True:
            limbs = [self.next_u64() for _ in range(4)]
            limbs[3] &= (1 << 63) - 1
            v = limbs[0] | (limbs[1] << 64) | (limbs[2] << 128) | (limbs[3] << 192)
            if v < R:
                return fr_from_mont_limbs(v)

    def state_digest(self):
        return self.h.copy().digest()


class InjectedChallenges:
    """Challenges independent of the transcript (for kernel-parity isolation)."""

    def __init__(self, seed):
        self.rng = SplitMix64(seed)

    def feed(self, data: bytes):
        pass

    def rand_fr(self):
        return self.rng.next_fr()
