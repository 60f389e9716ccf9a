"""The committed parity fixtures cannot drift from the oracle that made them: regenerating every
tests/golden/fixture_*.npz with tests/golden/make_fixtures.py gives the committed files byte for
byte (the writer fixes member timestamps and order)."""
import filecmp
import glob
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def test_fixtures_regenerate_byte_identical(tmp_path):
    spec = importlib.util.spec_from_file_location("make_fixtures", os.path.join(GOLDEN, "make_fixtures.py"))
    mf = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mf)
    mf.main(str(tmp_path))
    committed = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "fixture_*.npz")))
    made = sorted(os.path.basename(p) for p in glob.glob(os.path.join(str(tmp_path), "fixture_*.npz")))
    assert committed == made and len(made) == 5
    for name in made:
        assert filecmp.cmp(os.path.join(GOLDEN, name), os.path.join(str(tmp_path), name), shallow=False), name
