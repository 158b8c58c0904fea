"""The tuner's route decision (tools/tune.py pick_route / write_table), GPU-free: a rejected or
slower-than-default previous route must not survive a --merge, and of two routes that
time alike the more accurate one is written."""
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "boda-1_amd"))
sys.path.insert(0, ROOT)

from tools import tune  # noqa: E402

D = ("default", 0)


def test_fastest_admissible_route():
    med = {D: 10.0, ("a", 1): 8.0, ("b", 2): 9.0}
    assert tune.pick_route(med, {}, None, set(), 0.03) == ("a", 1)


def test_default_wins_gives_no_entry():
    med = {D: 8.0, ("a", 1): 9.0}
    assert tune.pick_route(med, {}, ("a", 1), set(), 0.03) is None


def test_rejected_previous_route_never_survives():
    med = {D: 10.0, ("wx43s10g", 0): 7.0}
    assert tune.pick_route(med, {}, ("wx43s10g", 0), {("wx43s10g", 0)}, 0.03) is None
    med[("gvs64x32w8", 1)] = 9.5
    assert tune.pick_route(med, {}, ("wx43s10g", 0), {("wx43s10g", 0)}, 0.03) == ("gvs64x32w8", 1)


def test_previous_route_kept_unless_beaten_by_min_gain():
    med = {D: 10.0, ("a", 1): 7.9, ("p", 3): 8.0}
    assert tune.pick_route(med, {}, ("p", 3), set(), 0.03) == ("p", 3)
    med[("a", 1)] = 7.0
    assert tune.pick_route(med, {}, ("p", 3), set(), 0.03) == ("a", 1)


def test_more_accurate_of_near_equal_routes():
    # dm3 at 6e-4 and gvs at 2e-4, within min_gain: gvs is written
    med = {D: 40.0, ("dm3w16x64c8", 1): 33.2, ("gvs64x32w8", 3): 33.9}
    err = {D: 2e-4, ("dm3w16x64c8", 1): 6e-4, ("gvs64x32w8", 3): 2e-4}
    assert tune.pick_route(med, err, None, set(), 0.03) == ("gvs64x32w8", 3)
    # outside min_gain the faster one stays
    med[("gvs64x32w8", 3)] = 36.0
    assert tune.pick_route(med, err, None, set(), 0.03) == ("dm3w16x64c8", 1)
    # an error less than 2x better does not move the pick
    med[("gvs64x32w8", 3)] = 33.9
    err[("gvs64x32w8", 3)] = 4e-4
    assert tune.pick_route(med, err, None, set(), 0.03) == ("dm3w16x64c8", 1)


def test_merge_deletes_entries(tmp_path):
    out = tmp_path / "t.tune"
    out.write_text("# header\n"
                   "conv 1 2 3 3 4 3 3 1 1 1 1 cfg=wx43s10g splits=0 red=i\n"
                   "conv 5 2 3 3 4 1 1 1 1 0 0 cfg=gvs16x16w8 splits=1 red=i\n")
    args = types.SimpleNamespace(out=str(out), merge=True, json="")
    table = {"conv 1 2 3 3 4 3 3 1 1 1 1": None,
             "conv 20 2 3 3 4 1 1 1 1 0 0": ("kn32p32c32q3w8", 2, 0.01, 0.02, 1)}
    tune.write_table(args, "plat", table, [])
    lines = [l for l in out.read_text().splitlines() if not l.startswith("#")]
    assert lines == ["conv 5 2 3 3 4 1 1 1 1 0 0 cfg=gvs16x16w8 splits=1 red=i",
                     "conv 20 2 3 3 4 1 1 1 1 0 0 cfg=kn32p32c32q3w8 splits=2 red=i wt=1"]


def test_import_leaves_the_table_alone():
    """Importing the tuner must not point BH_TUNE_FILE away from the committed table: pytest imports
    this module while collecting, and every GPU test of the same process would then run the heuristic
    routes instead of the table's (as one round-6 suite run did)."""
    assert os.environ.get("BH_TUNE_FILE") != "/nonexistent"
