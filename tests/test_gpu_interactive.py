"""The reference's round-level prover API (src/ahp/prover.rs:109-281) through the C ABI
(spx_prover_*), driven exactly as the reference's own interactive test drives it
(src/ahp/tests.rs:8-70: log_n 8, log_v 2, the TestSynthesizer circuit, verifier coins from an
external RNG). Every prover message must equal the Python oracle's message of the same round under
the same coins (oracle/py/spartan.py, whose prove() takes the challenge source as an argument), the
concatenation must equal the C oracle's injected-challenge proof, and the product's verifier must
accept it. Also the linear-sumcheck round entry spx_sumcheck_round against the oracle's
MLSumcheckProver.prove_round."""
import random

import pytest

pytestmark = pytest.mark.gpu

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


class Coins:
    """external verifier coins: SplitMix64 Fr draws (the oracle's injected-challenge source), and a
    record of what the prover sends"""

    def __init__(self, seed):
        from gen import SplitMix64

        self.rng = SplitMix64(seed)
        self.msgs = []

    def feed(self, data):
        self.msgs.append(bytes(data))

    def rand_fr(self):
        return self.rng.next_fr()

    def take(self, k):
        return [self.rand_fr() for _ in range(k)]


def _oracle_run(oc, inst, ppc, seed):
    """the Python oracle's prove with external coins: its messages in round order, and pm6"""
    import spartan

    pk = spartan.index(*[M.to_rows() for M in inst.mats])
    pp = spartan.PublicParameter.deserialize_uncompressed(ppc.serialize())
    z = inst.z_bytes
    vals = [int.from_bytes(z[32 * i : 32 * i + 32], "little") for i in range(len(z) // 32)]
    nv = len(inst.v_bytes) // 32
    fs = Coins(seed)
    proof = spartan.prove(pk, vals[:nv], vals[nv:], pp, fs=fs)
    return fs.msgs[4:], proof.pm6_bytes(), proof.to_bytes()  # the first 4 feeds absorb A, B, C, v


def _drive(spx, pk, inst, pp, seed, log_n, log_v):
    """ahp/tests.rs:22-63 with the product's round-level prover"""
    coins = Coins(seed)
    p = spx.InteractiveProver(pk, inst.v_bytes, inst.w_bytes)
    msgs = [p.prover_first_round(pp)]
    msgs.append(p.prover_second_round(coins.take(log_v), pp))
    msgs.append(p.prover_third_round(coins.take(log_n)))
    ch = None
    for _ in range(log_n):
        msgs.append(p.prove_first_sumcheck_round(ch))
        ch = coins.rand_fr()
    msgs.append(p.prove_fourth_round(ch))
    msgs.append(p.prove_fifth_round(*coins.take(3)))
    ch = None
    for _ in range(log_n):
        msgs.append(p.prove_second_sumcheck_round(ch))
        ch = coins.rand_fr()
    pm6 = p.prove_sixth_round(ch, pp)
    p.close()
    return msgs, pm6


@pytest.mark.parametrize("kind,log_n,log_v,param", [(1, 8, 2, 1), (0, 6, 3, 0), (3, 10, 4, 0)])
def test_interactive_rounds_match_oracle(spx, ctx, oc, kind, log_n, log_v, param):
    inst = oc.Instance(kind, log_n, log_v, 0x5EED0000 + log_n, param)
    pp = spx.MLProofForR1CS.setup(ctx, log_n, 77 + log_n)  # GPU keygen: its VerifierParameter is known
    ppc = oc.PP.load(pp.serialize_uncompressed())
    pk = spx.MLArgumentForR1CS.index(ctx, *[spx.Csr(M.n, M.row_ptr, M.col, M.val) for M in inst.mats])
    seed = 99 + log_n
    msgs, pm6 = _drive(spx, pk, inst, pp, seed, log_n, log_v)
    want_msgs, want_pm6, want_proof = _oracle_run(oc, inst, ppc, seed)
    assert len(msgs) == len(want_msgs) == 3 + log_n + 2 + log_n
    for i, (g, w) in enumerate(zip(msgs, want_msgs)):
        assert g == w, "message %d differs from the oracle's" % i
    assert pm6 == want_pm6
    # the messages in Proof field order (proof.rs:10-20): the sumchecks' Vec<ProverMsg> carry u64 counts
    L = log_n.to_bytes(8, "little")
    proof = b"".join(msgs[:3]) + L + b"".join(msgs[3 : 3 + log_n]) + b"".join(msgs[3 + log_n : 5 + log_n]) + L + \
        b"".join(msgs[5 + log_n :]) + pm6
    assert proof == want_proof == oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, ppc, 1, seed)
    # the whole-proof path with the same (injected) coins gives the same bytes, and verifies
    assert spx.MLArgumentForR1CS.prove(pk, inst.v_bytes, inst.w_bytes, pp, mode="injected", seed=seed) == proof
    assert spx.MLArgumentForR1CS.verify(pk, inst.v_bytes, proof, spx.verifier_parameter(pp), mode="injected", seed=seed)


def test_interactive_errors(spx, ctx, oc):
    log_n, log_v = 6, 2
    inst = oc.Instance(0, log_n, log_v, 31)
    ppc = oc.PP.keygen(log_n, 5)
    pp = spx.PublicParameter.load(ctx, ppc.serialize())
    pk = spx.MLArgumentForR1CS.index(ctx, *[spx.Csr(M.n, M.row_ptr, M.col, M.val) for M in inst.mats])
    # prover_init's checks (prover.rs:114-119)
    with pytest.raises(spx.InvalidArgument):
        spx.InteractiveProver(pk, inst.v_bytes[:96], inst.w_bytes)
    with pytest.raises(spx.InvalidArgument):
        spx.InteractiveProver(pk, inst.v_bytes, inst.w_bytes[:-32])
    p = spx.InteractiveProver(pk, inst.v_bytes, inst.w_bytes)
    with pytest.raises(spx.InvalidArgument):  # out of order
        p.prover_third_round([1] * log_n)
    p.prover_first_round(pp)
    with pytest.raises(spx.InvalidArgument):  # r_v of the wrong length
        p.prover_second_round([1] * (log_v + 1), pp)
    p.prover_second_round([3] * log_v, pp)
    p.prover_third_round([5] * log_n)
    with pytest.raises(spx.SumCheckError):  # "first round should be prover first"
        p.prove_first_sumcheck_round(7)
    p.prove_first_sumcheck_round(None)
    with pytest.raises(spx.SumCheckError):  # "verifier message is empty"
        p.prove_first_sumcheck_round(None)
    with pytest.raises(spx.SerializationError):  # a non-canonical coin
        p.prove_first_sumcheck_round(R.to_bytes(32, "little"))
    with pytest.raises(spx.InvalidArgument):  # the fourth round before the last sumcheck round
        p.prove_fourth_round(9)
    p.close()  # freed mid-way: the worker waiting for a coin is cancelled
    # a fresh session on the same context still proves correctly
    msgs, pm6 = _drive(spx, pk, inst, pp, 1234, log_n, log_v)
    assert pm6 == _oracle_run(oc, inst, ppc, 1234)[1]


def test_interactive_claims_context_and_fourth_round_retry(spx, ctx, oc):
    """a session owns its context's streams and tables until its worker's prove() returns: a prove, a
    verify or a second session on that context is refused (SPX_INVALID_ARGUMENT) instead of
    overwriting them; a non-canonical coin in the fourth round leaves the session retryable"""
    log_n, log_v = 6, 2
    inst = oc.Instance(0, log_n, log_v, 41)
    pp = spx.MLProofForR1CS.setup(ctx, log_n, 43)
    ppc = oc.PP.load(pp.serialize_uncompressed())
    pk = spx.MLArgumentForR1CS.index(ctx, *[spx.Csr(M.n, M.row_ptr, M.col, M.val) for M in inst.mats])
    seed = 4242
    coins = Coins(seed)
    p = spx.InteractiveProver(pk, inst.v_bytes, inst.w_bytes)
    with pytest.raises(spx.InvalidArgument):  # the context is claimed from prover_init on
        spx.MLArgumentForR1CS.prove(pk, inst.v_bytes, inst.w_bytes, pp)
    with pytest.raises(spx.InvalidArgument):
        spx.InteractiveProver(pk, inst.v_bytes, inst.w_bytes)
    msgs = [p.prover_first_round(pp), p.prover_second_round(coins.take(log_v), pp),
            p.prover_third_round(coins.take(log_n))]
    with pytest.raises(spx.InvalidArgument):  # mid-session: the worker holds the tables
        spx.MLArgumentForR1CS.prove(pk, inst.v_bytes, inst.w_bytes, pp)
    ch = None
    for _ in range(log_n):
        msgs.append(p.prove_first_sumcheck_round(ch))
        ch = coins.rand_fr()
    with pytest.raises(spx.SerializationError):  # non-canonical last point of r_x
        p.prove_fourth_round(R.to_bytes(32, "little"))
    msgs.append(p.prove_fourth_round(ch))  # the retry is accepted
    msgs.append(p.prove_fifth_round(*coins.take(3)))
    ch = None
    for _ in range(log_n):
        msgs.append(p.prove_second_sumcheck_round(ch))
        ch = coins.rand_fr()
    pm6 = p.prove_sixth_round(ch, pp)
    want_msgs, want_pm6, _ = _oracle_run(oc, inst, ppc, seed)
    assert msgs == want_msgs and pm6 == want_pm6
    # the worker has finished: the context is free again while the session object still exists
    proof = spx.MLArgumentForR1CS.prove(pk, inst.v_bytes, inst.w_bytes, pp)
    assert proof == oc.prove(inst.mats, inst.v_bytes, inst.w_bytes, ppc, 0, 0)
    p.close()


@pytest.mark.parametrize("log_n", [1, 2, 6, 13])
def test_sumcheck_round_entry(spx, ctx, log_n):
    import spartan

    rs = random.Random(log_n)
    n = 1 << log_n
    f = [rs.randrange(R) for _ in range(n)]
    g = [rs.randrange(R) for _ in range(n)]
    o = spartan.MLSumcheckProver([[f, g]], log_n)
    ev, _, _ = spx.sumcheck_round(ctx, f, g)
    assert [int.from_bytes(e, "little") for e in ev] == o.prove_round(None)
    if log_n < 2:
        return
    r = rs.randrange(R)
    ev, fo, go = spx.sumcheck_round(ctx, f, g, r)
    assert [int.from_bytes(e, "little") for e in ev] == o.prove_round(r)
    assert spx.fr_ints(fo) == spartan.fix_first(f, r) and spx.fr_ints(go) == spartan.fix_first(g, r)
