"""CPU: pin the oracle (the checker) before trusting it.

- against the reference's own known-answer tests (test/mpi/ccl/*.java, tests/golden/ccl_kat.json)
- against hand-derived Java-semantics vectors (tests/golden/java_semantics.json)
- against numpy for the wrap-around integer arithmetic of every integral type
- the worker validity table (src/mpi/<Op>Worker.java)
- the reference's documented defects in faithful mode
"""
import json
import os

import numpy as np
import pytest

import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TYPES = {v: k for k, v in O.TYPE_NAMES.items()}
OPS = {v: k for k, v in O.OP_NAMES.items()}


def _val(type_, x):
    if type_ in (O.FLOAT, O.DOUBLE):
        return float(x) if isinstance(x, str) else float(x)
    return int(x)


@pytest.mark.parametrize("case", json.load(open(os.path.join(GOLDEN, "java_semantics.json"))),
                         ids=lambda c: f"{c['op']}-{c['type']}-{c['in']}-{c['acc']}")
def test_java_semantics_vectors(case):
    t, op = TYPES[case["type"]], OPS[case["op"]]
    dt = O.NP_DTYPE[t]
    acc = np.array([_val(t, case["acc"])] * 3, dtype=dt)
    inp = np.array([_val(t, case["in"])] * 3, dtype=dt)
    exp = np.array([_val(t, case["expect"])] * 3, dtype=dt)
    got = O.apply(op, t, acc, inp)
    if t in (O.FLOAT, O.DOUBLE) and np.isnan(exp).all():
        assert np.isnan(got).all()
    else:
        assert np.array_equal(got.view(np.uint8), exp.view(np.uint8)), (case, got)


def test_reference_ccl_kats():
    for c in json.load(open(os.path.join(GOLDEN, "ccl_kat.json"))):
        P = c["P"]
        if c["test"] in ("allreduce_maxloc", "allreduce_minloc"):
            t = TYPES[c["type"]]
            op = OPS[c["op"]]
            sends = []
            for r in range(P):
                a = np.zeros(c["count"], O.NP_DTYPE[t])
                a["v"] = r + np.arange(c["count"])
                a["l"] = r
                sends.append(a)
            for flags in (0, O.FLAG_OLD):
                for x in O.allreduce(sends, c["count"], t, op, flags=flags):
                    assert [[int(v), int(lc)] for v, lc in zip(x["v"], x["l"])] == c["expect"], (c, flags)
            continue
        if c["test"] == "reduce_scatter":
            j = c["recvcount"]
            sends = [np.arange(j * P, dtype=np.int32)] * P
            for flags in (0, O.FLAG_OLD):
                got, _ = O.reduce_scatter(sends, [j] * P, O.INT, O.SUM, flags=flags)
                for r in range(P):
                    assert np.array_equal(got[r], P * (r * j + np.arange(j))), (c, flags)
            continue
        j = c["count"]
        sends = [np.arange(j, dtype=np.int32)] * P
        k = np.arange(j)
        for flags in (0, O.FLAG_OLD):
            if c["test"] == "allreduce":
                for r, x in enumerate(O.allreduce(sends, j, O.INT, O.SUM, flags=flags)):
                    assert np.array_equal(x, k * P), c
                    if isinstance(c["expect"], list):
                        assert x.tolist() == c["expect"]
            elif c["test"] == "reduce":
                x = O.reduce(sends, j, O.INT, O.SUM, c["root"], flags=flags)[c["root"]]
                assert np.array_equal(x, k * P), c
            elif c["test"] == "reduce2":
                x = O.reduce(sends, j, O.INT, O.PROD, c["root"], flags=flags)[c["root"]]
                assert np.array_equal(x, k * k), c
            elif c["test"] == "scan":
                for r, x in enumerate(O.scan(sends, j, O.INT, O.SUM, flags=flags)):
                    assert np.array_equal(x, k * (r + 1)), c


@pytest.mark.parametrize("type_", [O.BYTE, O.SHORT, O.CHAR, O.INT, O.LONG])
def test_integer_wrap_matches_numpy(type_):
    rng = np.random.default_rng(type_)
    dt = O.NP_DTYPE[type_]
    info = np.iinfo(dt)
    a = rng.integers(info.min, info.max, 5000, dtype=dt, endpoint=True)
    b = rng.integers(info.min, info.max, 5000, dtype=dt, endpoint=True)
    with np.errstate(over="ignore"):
        ref = {O.SUM: b + a, O.PROD: b * a, O.BAND: b & a, O.BOR: b | a, O.BXOR: b ^ a,
               O.MAX: np.where(b > a, b, a), O.MIN: np.where(b < a, b, a)}
    for op, exp in ref.items():
        got = O.apply(op, type_, a.copy(), b)
        assert np.array_equal(got, exp), O.OP_NAMES[op]


def test_float_max_min_compare_form():
    a = np.array([1.0, np.nan, 0.0, -0.0, -np.inf], dtype=np.float64)
    b = np.array([np.nan, 2.0, -0.0, 0.0, np.nan], dtype=np.float64)
    mx = O.apply(O.MAX, O.DOUBLE, a.copy(), b)  # acc = a, in = b
    assert mx[0] == 1.0 and np.isnan(mx[1]) and not np.signbit(mx[2]) and np.signbit(mx[3])
    assert mx[4] == -np.inf


def test_loc_tie_rule_and_nan():
    """MAXLOC/MINLOC: strict compare moves (value, index); equal values keep the smaller index; a
    NaN value never wins; -0/+0 tie keeps acc's value but may lower the index."""
    t = O.DOUBLE2
    acc = np.zeros(5, O.NP_DTYPE[t])
    inp = np.zeros(5, O.NP_DTYPE[t])
    acc["v"] = [1.0, 2.0, np.nan, 0.0, 5.0]
    acc["l"] = [7, 3, 4, 9, 1]
    inp["v"] = [3.0, 2.0, 8.0, -0.0, np.nan]
    inp["l"] = [1, 1, 0, 2, 0]
    mx = O.apply(O.MAXLOC, t, acc.copy(), inp)
    assert mx["v"][0] == 3.0 and mx["l"][0] == 1          # strictly greater: both move
    assert mx["v"][1] == 2.0 and mx["l"][1] == 1          # tie: smaller index
    assert np.isnan(mx["v"][2]) and mx["l"][2] == 4       # NaN acc never replaced
    assert not np.signbit(mx["v"][3]) and mx["l"][3] == 2  # +0 kept, index lowered
    assert mx["v"][4] == 5.0 and mx["l"][4] == 1          # NaN in never wins
    assert O.check(O.MAXLOC, O.INT) == 1 and O.check(O.SUM, O.INT2) == 1 and O.check(O.MINLOC, O.FLOAT2) == 0


def test_worker_table():
    """46 typed classes: SUM/PROD/MAX/MIN x 7 numeric types, BAND/BOR/BXOR x 5 integral, L* x boolean."""
    pairs = set(O.valid_pairs())
    assert len(pairs) == 46
    assert (O.SUM, O.BOOLEAN) not in pairs and (O.BAND, O.DOUBLE) not in pairs
    assert (O.LAND, O.INT) not in pairs and (O.LXOR, O.BOOLEAN) in pairs
    assert O.check(O.SUM, 9) == 2  # PACKED: no worker


def test_mst_float_order_p6():
    """P=6 root 0 order (((x4+x3)+x5)+(x2+(x1+x0))) — grouping matters for floats."""
    xs = [np.array([v], dtype=np.float32) for v in (1e8, 1.0, -1e8, 3.0, 1e-3, 7.0)]
    got = O.reduce(xs, 1, O.FLOAT, O.SUM, 0)[0]
    f = np.float32
    exp = ((f(1e-3) + f(3.0)) + f(7.0)) + (f(-1e8) + (f(1.0) + f(1e8)))
    assert got[0] == exp


def test_faithful_defects():
    P = 3
    rng = np.random.default_rng(0)
    s = [rng.integers(0, 100, 6).astype(np.int32) for _ in range(P)]
    # A3: BOR/BXOR never combine -> Allreduce returns rank 0's input everywhere, Scan returns own
    for r, x in enumerate(O.allreduce(s, 6, O.INT, O.BXOR, flags=O.FLAG_FAITHFUL)):
        assert np.array_equal(x, s[0])
    for r, x in enumerate(O.scan(s, 6, O.INT, O.BOR, flags=O.FLAG_FAITHFUL)):
        assert np.array_equal(x, s[r])
    # A9: BKT SUM block r = x_r + (P-1) x_{r+1}; PROD/BAND all zeros
    got, _ = O.reduce_scatter(s, [2] * P, O.INT, O.SUM, flags=O.FLAG_FAITHFUL)
    for r in range(P):
        b = slice(2 * r, 2 * r + 2)
        assert np.array_equal(got[r], s[r][b] + (P - 1) * s[(r + 1) % P][b])
    for op in (O.PROD, O.BAND):
        got, _ = O.reduce_scatter(s, [2] * P, O.INT, op, flags=O.FLAG_FAITHFUL)
        assert all((g == 0).all() for g in got)
    # MPI mode is the correct reduction
    got, _ = O.reduce_scatter(s, [2] * P, O.INT, O.SUM)
    tot = sum(s)
    for r in range(P):
        assert np.array_equal(got[r], tot[2 * r:2 * r + 2])


def test_ft_allreduce_orders_differ_per_rank():
    """FT_Allreduce (old collectives): rank r starts from x_r — float results may differ per rank."""
    xs = [np.array([v], dtype=np.float32) for v in (1e8, 1.0, -1e8, 1.0)]
    res = O.allreduce(xs, 1, O.FLOAT, O.SUM, flags=O.FLAG_OLD)
    f = np.float32
    for r in range(4):
        acc = xs[r][0]
        for i in range(4):
            if i != r:
                acc = f(xs[i][0] + acc)
        assert res[r][0] == acc


def test_cpu_baseline_timers_run():
    t = O.time_combine(O.SUM, O.DOUBLE, 1 << 16, 3)
    assert 0 < t < 1
    t = O.time_allreduce_mst(4, 1 << 14, 3, pin=False)
    assert 0 < t < 5


# ---- the first reference-produced floating-point result on the path (JGF SparseMatmult) --------

JGF = json.load(open(os.path.join(GOLDEN, "jgf_sparsematmult.json")))


@pytest.mark.parametrize("kat", JGF["java_random_kat"], ids=lambda k: f"{k['seed']}-{k['call']}")
def test_java_random_known_answers(kat):
    """java.util.Random restated from the Java API's LCG; the published first outputs of seeds 42, 0."""
    r = O.JavaRandom(kat["seed"])
    assert getattr(r, kat["call"])() == kat["expect"]


@pytest.mark.parametrize("size", ["A", "B", "C"])
def test_jgf_sparsematmult_refval_exact_p1(size):
    """JGFSparseMatmultBench.java:148: at P = 1 the Allreduce is an identity, so the oracle's input
    generation + 200 reps of SparseMatmult.java:241-246 must give the reference's refval to the bit."""
    assert O.jgf_sparse_matmult(1, size=size) == JGF["sizes"][size]["refval"]


@pytest.mark.parametrize("flags", [0, O.FLAG_OLD], ids=["mst", "old_ft"])
@pytest.mark.parametrize("P", [2, 3, 4, 8])
def test_jgf_sparsematmult_refval_tolerance(P, flags):
    """At P > 1 the Allreduce regroups the per-rank partial sums; the reference's own check is
    |ytotal - refval| <= 1e-12 (JGFSparseMatmultBench.java:149-150)."""
    got = O.jgf_sparse_matmult(P, flags=flags)
    assert abs(got - JGF["sizes"]["A"]["refval"]) <= JGF["tolerance"], got


def test_topo_map_kat():
    """test/mpi/topo/map.java:63-79 (tests/golden/map_kat.json): Reduce INT SUM of one-hot rows."""
    k = json.load(open(os.path.join(GOLDEN, "map_kat.json")))
    P = k["P"]
    sends = [(np.arange(P) == r).astype(np.int32) for r in range(P)]  # new_rank = rank
    for flags in (0, O.FLAG_OLD, O.FLAG_FAITHFUL):
        got = O.reduce(sends, k["count"], O.INT, O.SUM, k["root"], flags=flags)[k["root"]]
        assert got.tolist() == k["expect"], flags


# ---- JGF MolDyn: in-place Allreduce(DOUBLE, SUM) every move, reference-held kinetic energy -------

MD = json.load(open(os.path.join(GOLDEN, "jgf_moldyn.json")))


def test_java_log_is_fdlibm():
    """StrictMath.log (fdlibm 5.3), restated in oracle/jgf_moldyn.c: exact on the points where a
    log is exactly representable, and within one ulp of the correctly rounded value elsewhere."""
    L = O.lib()
    assert L.ora_java_log(1.0) == 0.0
    assert L.ora_java_log(2.0) == np.log(2.0)
    assert L.ora_java_log(0.5) == -np.log(2.0)
    rng = np.random.default_rng(7)
    for x in rng.uniform(1e-6, 1.0, 2000):
        assert abs(L.ora_java_log(x) - np.log(x)) <= np.spacing(abs(np.log(x))), x


@pytest.mark.parametrize("size", ["A", "B"])
def test_jgf_moldyn_refval_exact_p1(size):
    """JGFMolDynBench.java:72: at P = 1 every Allreduce is an identity, so the oracle's restatement of
    md.java (with fdlibm's log, the one StrictMath specifies) must end on the reference's kinetic energy
    to the bit after 50 chaotic moves."""
    ek, _ = O.jgf_moldyn(1, size=size)
    assert ek == MD["sizes"][size]["refval"]


@pytest.mark.parametrize("flags", [0, O.FLAG_OLD], ids=["mst", "old_ft"])
@pytest.mark.parametrize("P", [2, 3, 4, 8])
def test_jgf_moldyn_regrouped_sums(P, flags):
    """At P > 1 the Allreduce regroups the per-rank partial forces; the dynamics are chaotic, so the
    last bits of ek move. This test allows 1.4e-12 (6 ulps), looser than the reference's own 1e-12 check
    (JGFMolDynBench.java:73): by THIS restatement the MST order misses 1e-12 at P = 4 and 8. That is an
    unverified claim about the reference (no JVM here to run it at P > 1), not a finding; the bit-exact
    pins are P = 1 (refval itself) and, at every P, GPU == oracle (test_jgf_moldyn_refval). The integer
    interaction count — never reset, summed over ranks every move — wraps like a Java int and agrees on
    every rank."""
    ek, inter = O.jgf_moldyn(P, flags=flags)
    assert abs(ek - MD["sizes"]["A"]["refval"]) <= 1.4e-12, ek
    assert len(set(inter)) == 1


@pytest.mark.parametrize("P", [2, 3, 4, 8])
def test_microbenchmark_max_pattern(P):
    """test/microbenchmarkmpiJava/{allreduce,reduce,reducescatter,scan}: every rank sends A[i] = 1/(i+1)
    with MPI.MAX — the result is A (MAX of equal values keeps the accumulator), in MPI and in faithful
    mode (the BKT ring's defect is invisible on identical positive inputs: max(x, x, 0) = x)."""
    n = 1000 * P
    A = 1.0 / (np.arange(n) + 1.0)
    for flags in (0, O.FLAG_OLD, O.FLAG_FAITHFUL):
        for x in O.allreduce([A] * P, n, O.DOUBLE, O.MAX, flags=flags):
            assert np.array_equal(x, A)
        assert np.array_equal(O.reduce([A] * P, n, O.DOUBLE, O.MAX, 0, flags=flags)[0], A)
        for r, x in enumerate(O.scan([A] * P, n, O.DOUBLE, O.MAX, flags=flags)):
            assert np.array_equal(x, A)
        got, _ = O.reduce_scatter([A] * P, [1000] * P, O.DOUBLE, O.MAX, flags=flags)
        for r in range(P):
            assert np.array_equal(got[r], A[1000 * r:1000 * (r + 1)])


# ---- JGF RayTracer: in-place Reduce(DOUBLE, SUM, root 0) of the pixel checksum, exact ---------------

RT = json.load(open(os.path.join(GOLDEN, "jgf_raytracer.json")))


@pytest.mark.parametrize("size", ["A", "B"])
def test_jgf_raytracer_checksum_is_refval(size):
    """JGFRayTracerBench.java:87-88: the oracle's restatement of the renderer (oracle/jgf_raytracer.c,
    the reference's shared temporary ray included) gives the reference's pixel checksum exactly for
    both sizes — a rendering of 22,500 / 250,000 pixels through up to 255 rays each."""
    rows = O.jgf_raytracer_rows(size)
    assert rows.size == RT["sizes"][size]["width"]
    assert int(rows.sum()) == RT["sizes"][size]["refval"]


@pytest.mark.parametrize("flags", [0, O.FLAG_OLD, O.FLAG_FAITHFUL], ids=["mst", "old_ft", "faithful"])
@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 8, 13])
def test_jgf_raytracer_reduce_every_P(P, flags):
    """RayTracer.java:275-279: each rank's partial checksum (its rows y = rank, rank + P, ...) goes into
    an in-place Reduce(DOUBLE, SUM, root 0); the partials are integers below 2^53, so the reduction is
    exact in every order and rank 0 holds refval at EVERY P — a reference-held Reduce result on DOUBLE."""
    parts = O.jgf_raytracer_partials(P, "A")
    assert len(parts) == P and all(float(p[0]).is_integer() for p in parts)
    assert O.jgf_raytracer(P, flags=flags) == RT["sizes"]["A"]["refval"]
