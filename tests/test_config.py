"""Host-side config handling (parent merge, comments) mirroring src/testbed.cu:95-106,228-314."""
import json


def test_merge_patch_and_parent(tmp_path):
    from __graft_entry__ import load_package
    pkg = load_package()
    (tmp_path / "base.json").write_text('{"a": {"b": 1, "c": 2}, // comment\n "d": [1,2], }')
    (tmp_path / "child.json").write_text(json.dumps({"parent": "base.json", "a": {"c": 3}, "d": None}))
    cfg = pkg.load_config(str(tmp_path / "child.json"))
    assert cfg == {"a": {"b": 1, "c": 3}}


def test_nerf_config_variants():
    from __graft_entry__ import load_package
    pkg = load_package()
    c2 = pkg.nerf_config("C2")
    assert c2["encoding"]["n_levels"] == 4 and c2["encoding"]["n_features_per_level"] == 4
    assert c2["encoding"]["per_level_scale"] == 2.0
    c2p = pkg.nerf_config("C2p")
    assert c2p["encoding"]["n_levels"] == 16 and c2p["encoding"]["n_features_per_level"] == 2
