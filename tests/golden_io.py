"""Readers for the committed golden fixtures (tests/golden/<variant>/)."""
import gzip
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def variants():
    return sorted(d for d in os.listdir(GOLDEN)
                  if os.path.isfile(os.path.join(GOLDEN, d, "meta.json")))


def meta(name):
    with open(os.path.join(GOLDEN, name, "meta.json")) as f:
        return json.load(f)


def text(name, fn):
    with gzip.open(os.path.join(GOLDEN, name, fn + ".gz"), "rb") as f:
        return f.read()


def int_table(name, fn):
    rows = [l for l in text(name, fn).decode().splitlines() if l.strip()]
    return np.array([[int(x) for x in l.split(",")] for l in rows], dtype=np.int64)


# Fortran edit descriptors used by the reference's formatted writes
def fmt_i10(*cols):
    """(i10,",",i10,...) records, e.g. Square/bondc.f:604-605."""
    n = len(cols[0])
    fmt = ",".join(["%10d"] * len(cols)) + "\n"
    return "".join(fmt % tuple(int(c[i]) for c in cols) for i in range(n)).encode()
