"""The GPU tick *algorithm* (numpy model in tests/gpu_model.py) against the
golden vectors and the sequential oracle.  CPU only: validates the
decomposition the kernels implement, independent of HIP."""
import glob
import os

import numpy as np
import pytest

import gpu_model
from oracle import fixture_expect, fixture_ticks

GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "small_*.npz")))


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p)[:-4] for p in GOLDEN])
def test_model_matches_reference(path):
    z = np.load(path)
    st = dict(reg=z["init_reg"], free=z["init_free"], hb=z["init_hb"], epoch=z["init_epoch"],
              queue=z["init_queue"], log=z["init_log"])
    carried = 0
    for t, tk in enumerate(fixture_ticks(z)):
        exp = fixture_expect(z, t)
        n_pending = carried + tk["n_new"]
        out, st = gpu_model.tick(st, tk["now"], float(z["tte"]), tk["ev_kind"], tk["ev_slot"], tk["ev_val"],
                                 tk["ev_ts"], tk["ev_seq"], n_pending)
        for k in ("reconnect", "assign", "orphans", "evicted"):
            np.testing.assert_array_equal(out[k], exp[k], err_msg="tick %d %s" % (t, k))
        np.testing.assert_array_equal(st["queue"], exp["post_queue"])
        np.testing.assert_array_equal(st["reg"], exp["post_reg"])
        reg = exp["post_reg"].astype(bool)
        np.testing.assert_array_equal(st["free"][reg], exp["post_free"][reg])
        np.testing.assert_array_equal(st["hb"][reg], exp["post_hb"][reg])
        carried = n_pending + len(out["orphans"]) - len(out["assign"])
