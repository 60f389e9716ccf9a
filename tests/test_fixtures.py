"""The committed parity fixtures cannot drift from the oracle that made them: regenerating every
tests/golden/fixture_*.npz with tests/golden/make_fixtures.py gives the same members with equal
arrays (compared as arrays, loaded with allow_pickle=False: the deflate bytes depend on the zlib
build, the arrays do not)."""
import glob
import importlib.util
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def test_fixtures_regenerate_identical(tmp_path):
    spec = importlib.util.spec_from_file_location("make_fixtures", os.path.join(GOLDEN, "make_fixtures.py"))
    mf = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mf)
    mf.main(str(tmp_path))
    committed = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "fixture_*.npz")))
    made = sorted(os.path.basename(p) for p in glob.glob(os.path.join(str(tmp_path), "fixture_*.npz")))
    assert committed == made and len(made) == 8
    for name in made:
        with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as a, \
                np.load(os.path.join(str(tmp_path), name), allow_pickle=False) as b:
            assert sorted(a.files) == sorted(b.files), name
            for k in a.files:
                assert a[k].dtype == b[k].dtype and np.array_equal(a[k], b[k]), (name, k)
