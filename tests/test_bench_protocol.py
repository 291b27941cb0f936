"""bench.py's PMC bookkeeping (CPU): a stored profile fills a line's traffic / issue /
occupancy / L2 fields only when it was taken on the same workload, protocol, settings and
build, and its timed launches ran within 10% of the line's kernel time."""
import bench


def _ident(**kw):
    d = {"config": "c3", "order": None, "grid": None, "k": 4, "proposal": "pairs",
         "base": "base mu", "percent": 0.05, "seed": 0, "chains": 65536, "chain_id0": 0,
         "inner": 1000, "warmup": 5, "steps": 20, "resumed_steps": 0, "maps": False,
         "flipwalk_env": {}, "build": "src=0123456789abcdef flags=-O3"}
    d.update(kw)
    return d


def test_pmc_key_names_the_protocol():
    assert bench.pmc_key("c3", None, 65536, 1000, 5, 20) == "c3_65536_1000_w5_s20"
    assert bench.pmc_key("c3", None, 8192, 1000, 5, 20, 8192) == "c3_8192_1000_w5_s20_id8192"
    assert bench.pmc_key("c5", None, 8192, 1000, 10, 100, 0, 100000) == "c5_8192_1000_w10_s100_r100000"
    assert bench.pmc_key("c4", "random", 16384, 1000, 5, 20) == "c4r_16384_1000_w5_s20"
    assert bench.pmc_key("c4", "hilbert", 16384, 1000, 5, 20) == "c4_16384_1000_w5_s20"


def test_pmc_mismatch_accepts_only_the_same_run():
    prof = {"source": "profiles/r05/x", "identity": _ident(), "kernel_trace": {"avg_ms": 15.2}}
    assert bench.pmc_mismatch(prof, _ident(), 16.0) is None  # 5% apart
    assert "more than 10%" in bench.pmc_mismatch(prof, _ident(), 17.5)
    why = bench.pmc_mismatch(prof, _ident(build="src=ffffffffffffffff flags=-O3"), 15.2)
    assert why and "build" in why
    assert "flipwalk_env" in bench.pmc_mismatch(prof, _ident(flipwalk_env={"FLIPWALK_SPEC": "2"}), 15.2)
    assert "grid" in bench.pmc_mismatch(prof, _ident(grid=40), 15.2)
    assert "no PMC profile" in bench.pmc_mismatch(None, _ident(), 15.2)
    assert "no identity" in bench.pmc_mismatch({"source": "old"}, _ident(), 15.2)


def test_committed_profiles_match_the_in_tree_library():
    """Every stored profile is named by its own protocol and was taken with the library the
    tree ships, so the driver's lines use it: a kernel change without re-profiling fails
    here (on CPU), not silently as ``pmc.used: false`` in the round's bench line.  The
    driver's protocol (``--steps 20 --warmup 5``, C3, default launch length) must be among
    them."""
    import glob
    import json
    import os
    from flipcomplexityempirical_amd._lib import build_info

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    files = sorted(glob.glob(os.path.join(root, "profiles", "pmc", "*.json")))
    assert files, "no PMC profiles under profiles/pmc"
    build = build_info()
    for f in files:
        prof = json.load(open(f))
        ident = prof["identity"]
        key = bench.pmc_key(ident["config"], ident["order"], ident["chains"], ident["inner"],
                            ident["warmup"], ident["steps"], ident["chain_id0"],
                            ident["resumed_steps"])
        assert os.path.basename(f) == key + ".json", f
        assert ident["build"] == build, f"{f}: profiled build {ident['build']!r}, tree {build!r}"
        assert ident["flipwalk_env"] == {}, f
    keys = {os.path.basename(f)[:-5] for f in files}
    assert bench.pmc_key("c3", None, 65536, 5000, 5, 20) in keys
