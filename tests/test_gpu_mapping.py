"""The product's own id math (dccrgx_mapping.hpp, evaluated by a device
kernel through dccrgx_mapping_batch, and the host scalar queries) against the
reference's Mapping compiled as-is (tests/golden/mapping_ref.json, made by
tests/golden/make_golden.py from oracle/_ref/ref_probe): every id record and
every get_cell_from_indices query, bit-exact."""
import json
import os

import numpy as np
import pytest

import dccrg_amd

pytestmark = pytest.mark.gpu


def _grids(golden_dir):
    with open(os.path.join(golden_dir, "mapping_ref.json")) as f:
        return json.load(f)


def test_device_mapping_matches_reference(gpu, golden_dir):
    for gr in _grids(golden_dir):
        g = dccrg_amd.Dccrg(0, 1, 0)
        g.set_initial_length(gr["length"]).set_maximum_refinement_level(gr["max_ref_lvl"])
        assert g.get_last_cell() == gr["last_cell"]
        recs = gr["ids"]
        b = g.mapping_batch(np.array([r["id"] for r in recs], np.uint64))
        for i, r in enumerate(recs):
            assert b["level"][i] == r["level"], r
            if r["level"] < 0:
                continue
            assert b["indices"][i].tolist() == r["indices"], r
            assert int(b["length"][i]) == r["length"], r
            assert int(b["parent"][i]) == r["parent"], r
            assert int(b["child"][i]) == r["child"], r
            assert int(b["level0_parent"][i]) == r["level0_parent"], r
            assert b["siblings"][i].tolist() == r["siblings"], r
            assert g.get_refinement_level(r["id"]) == r["level"]
            assert list(g.get_indices(r["id"])) == r["indices"]
        for q in gr["queries"]:
            assert g.get_cell_from_indices(q["indices"], q["level"]) == q["cell"], q
        g.close()
