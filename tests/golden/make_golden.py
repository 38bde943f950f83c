"""Generate the golden fixtures under tests/golden/ (committed; rerun to regenerate).

1. ccl_kat.json — the reference's own known-answer tests, restated as data: inputs and expected
   outputs exactly as test/mpi/ccl/{allreduce,reduce,reduce2,scan,reduce_scatter,
   allreduce_maxminloc}.java build and check them (out[i] = i on every rank; expected k*tasks, k*k,
   k*(rank+1), tasks*(rank*j+k); MAXLOC (size-1+i, size-1), MINLOC (i, 0) for in = (rank+i, rank)).
   No code from the reference is copied; only the input formulas and asserted values.
2. java_semantics.json — single-element cases whose expected value follows from the Java Language
   Specification rules the typed Op classes rely on (narrowing after int promotion, two's-complement
   wrap, unsigned char, `if (a > b)` comparisons with NaN and signed zeros). Written by hand, not
   produced by the oracle, so they pin the oracle independently.
3. map_kat.json — test/mpi/topo/map.java's Reduce KAT (one-hot rows, INT SUM, every count 1).
4. jgf_sparsematmult.json, jgf_moldyn.json — the reference-held double results of the two JGF
   benchmarks whose kernels are Allreduce(DOUBLE, SUM) calls (refval, sizes, seeds, tolerances as data)
   and java.util.Random's published first outputs.
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def ccl_kats():
    cases = []
    for P in (1, 2, 3, 4, 8):
        for j in (1, 10, 100, 1000, 10000):
            cases.append({"test": "allreduce", "source": "test/mpi/ccl/allreduce.java:73-86",
                          "P": P, "count": j, "type": "INT", "op": "SUM",
                          "input": "out[i]=i", "expect": [k * P for k in range(j)] if j <= 100 else "k*tasks"})
            cases.append({"test": "reduce", "source": "test/mpi/ccl/reduce.java:73-87",
                          "P": P, "count": j, "type": "INT", "op": "SUM", "root": P // 2,
                          "input": "out[i]=i", "expect": "k*tasks"})
            cases.append({"test": "scan", "source": "test/mpi/ccl/scan.java:73-85",
                          "P": P, "count": j, "type": "INT", "op": "SUM",
                          "input": "out[i]=i", "expect": "k*(rank+1)"})
        cases.append({"test": "reduce2", "source": "test/mpi/ccl/reduce2.java:73-92",
                      "P": 2, "count": 1000, "type": "INT", "op": "PROD", "root": 1,
                      "input": "out[i]=i", "expect": "k*k"})
        for tname in ("SHORT2", "INT2", "LONG2", "FLOAT2", "DOUBLE2"):
            cases.append({"test": "allreduce_maxloc", "source": "test/mpi/ccl/allreduce_maxminloc.java:52-230",
                          "P": P, "count": 10, "type": tname, "op": "MAXLOC",
                          "input": "in[2i]=rank+i, in[2i+1]=rank",
                          "expect": [[P - 1 + i, P - 1] for i in range(10)]})
            cases.append({"test": "allreduce_minloc", "source": "test/mpi/ccl/allreduce_maxminloc.java:240-400",
                          "P": P, "count": 10, "type": tname, "op": "MINLOC",
                          "input": "in[2i]=rank+i, in[2i+1]=rank",
                          "expect": [[i, 0] for i in range(10)]})
        cases.append({"test": "reduce_scatter", "source": "test/mpi/ccl/reduce_scatter.java:81-96",
                      "P": P, "recvcount": 10, "type": "INT", "op": "SUM",
                      "input": "out[i]=i for i < 10*tasks", "expect": "tasks*(rank*10+k)"})
    return cases


# (op, type, in, acc, expected) — value of arr[i] after one perform with arr1[i] = in, arr[i] = acc.
# Floats as strings for nan/inf/-0.0; BOOLEAN as 0/1.
JAVA = [
    ("SUM", "BYTE", 127, 1, -128),              # (byte)(127 + 1)
    ("SUM", "BYTE", -128, -1, 127),
    ("SUM", "SHORT", 32767, 1, -32768),
    ("SUM", "CHAR", 65535, 1, 0),               # char is unsigned 16-bit
    ("SUM", "INT", 2147483647, 1, -2147483648),
    ("SUM", "LONG", 9223372036854775807, 1, -9223372036854775808),
    ("PROD", "CHAR", 65535, 65535, 1),           # int overflow, then (char) keeps the low 16 bits
    ("PROD", "BYTE", -128, -1, -128),            # (byte)(128)
    ("PROD", "SHORT", 300, 300, 24464),          # (short)90000
    ("PROD", "INT", 65536, 65536, 0),
    ("PROD", "LONG", 4294967296, 4294967296, 0),
    ("MAX", "CHAR", 65535, 1, 65535),            # unsigned compare
    ("MIN", "CHAR", 65535, 1, 1),
    ("MAX", "BYTE", -1, 1, 1),                   # signed compare
    ("MIN", "BYTE", -128, 127, -128),
    ("MAX", "DOUBLE", "nan", "1.0", "1.0"),     # NaN in never replaces (nan > 1 is false)
    ("MAX", "DOUBLE", "1.0", "nan", "nan"),     # NaN acc is never replaced (1 > nan is false)
    ("MIN", "FLOAT", "nan", "1.0", "1.0"),
    ("MAX", "DOUBLE", "-0.0", "0.0", "0.0"),    # tie keeps acc
    ("MAX", "DOUBLE", "0.0", "-0.0", "-0.0"),
    ("MIN", "FLOAT", "0.0", "-0.0", "-0.0"),
    ("MIN", "FLOAT", "-0.0", "0.0", "0.0"),
    ("SUM", "DOUBLE", "inf", "-inf", "nan"),
    ("SUM", "DOUBLE", "4.9e-324", "4.9e-324", "1e-323"),  # subnormals kept
    ("SUM", "FLOAT", "1.0", "1e-08", "1.0"),
    ("PROD", "FLOAT", "1e-30", "1e-30", "0.0"),
    ("BAND", "INT", -1, 12345, 12345),
    ("BOR", "SHORT", -32768, 1, -32767),
    ("BXOR", "LONG", -1, 0, -1),
    ("BXOR", "CHAR", 65535, 255, 65280),
    ("LAND", "BOOLEAN", 1, 0, 0),
    ("LAND", "BOOLEAN", 1, 1, 1),
    ("LOR", "BOOLEAN", 0, 0, 0),
    ("LOR", "BOOLEAN", 1, 0, 1),
    ("LXOR", "BOOLEAN", 1, 1, 0),
    ("LXOR", "BOOLEAN", 0, 1, 1),
]


def map_kat():
    """test/mpi/topo/map.java:52-79: 8 ranks, a 2x4 Cartcomm; Map() returns the rank itself
    (src/mpi/Cartcomm.java:496-516); sbuf[new_rank] = 1, Reduce(INT, SUM, root 0), rbuf[i] == 1."""
    return {"test": "topo_map", "source": "test/mpi/topo/map.java:63-79", "P": 8, "count": 8,
            "type": "INT", "op": "SUM", "root": 0, "new_rank": "Cartcomm.Map = rank (Cartcomm.java:515)",
            "input": "sbuf[i] = (i == new_rank)", "expect": [1] * 8}


def jgf_sparsematmult():
    """The reference-held double results of the JGF SparseMatmult benchmark, whose kernel is 200
    Allreduce(DOUBLE, SUM) calls (SparseMatmult.java:239-247). Values copied as data from
    JGFSparseMatmultBench.java; java.util.Random known answers from the Java API's specified LCG
    (they are the widely published outputs for seeds 42 and 0)."""
    return {
        "source": "test/jgf_mpj_benchmarks/section2/sparsematmult/JGFSparseMatmultBench.java",
        "seed": 10101010, "iterations": 200, "tolerance": 1.0e-12, "tolerance_source": ":150",
        "sizes": {"A": {"M": 50000, "N": 50000, "nz": 250000, "refval": 75.02484945753453},
                  "B": {"M": 100000, "N": 100000, "nz": 500000, "refval": 150.0130719633895},
                  "C": {"M": 500000, "N": 500000, "nz": 2500000, "refval": 749.5245870753752}},
        "refval_source": ":148",
        "java_random_kat": [{"seed": 42, "call": "nextInt", "expect": -1170105035},
                            {"seed": 0, "call": "nextDouble", "expect": 0.730967787376657},
                            {"seed": 0, "call": "nextInt", "expect": -1155484576}],
    }


def jgf_moldyn():
    """The reference-held results of the JGF MolDyn benchmark, whose every move ends in in-place
    Allreduce(DOUBLE, SUM) of the partial forces, epot, vir and an Allreduce(INT, SUM) (md.java:248-264).
    Values copied as data from JGFMolDynBench.java:72-73."""
    return {"source": "test/jgf_mpj_benchmarks/section3/moldyn/JGFMolDynBench.java", "refval_source": ":72",
            "tolerance": 1.0e-12, "tolerance_source": ":73", "moves": 50, "moves_source": "md.java:77",
            "sizes": {"A": {"mm": 8, "mdsize": 2048, "refval": 1731.4306625334357},
                      "B": {"mm": 13, "mdsize": 8788, "refval": 7397.392307839352}}}


def main():
    with open(os.path.join(HERE, "ccl_kat.json"), "w") as f:
        json.dump(ccl_kats(), f, indent=0)
    with open(os.path.join(HERE, "map_kat.json"), "w") as f:
        json.dump(map_kat(), f, indent=1)
    with open(os.path.join(HERE, "jgf_sparsematmult.json"), "w") as f:
        json.dump(jgf_sparsematmult(), f, indent=1)
    with open(os.path.join(HERE, "jgf_moldyn.json"), "w") as f:
        json.dump(jgf_moldyn(), f, indent=1)
    with open(os.path.join(HERE, "java_semantics.json"), "w") as f:
        json.dump([dict(zip(("op", "type", "in", "acc", "expect"), r)) for r in JAVA], f, indent=1)


if __name__ == "__main__":
    main()
