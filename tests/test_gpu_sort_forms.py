"""Both forms of the hand-written MSM bucket sort (msm_common.hip: the LDS-staged form chosen for
dense batches, the direct form for a sharded rank's sparse ones), each forced for a whole child
process by SPX_SORT_FORM, and the MSM's A/B knobs (SPX_MSM_LEVELS=0: no XYZZ partial level, the
weighting leaf adds every partial; SPX_MSM_SEG1=8: short accumulation segments, many partials), each
against the oracle byte for byte (tests/sort_form_check.py)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("setting", ["SPX_SORT_FORM=staged", "SPX_SORT_FORM=direct", "SPX_MSM_LEVELS=0",
                                     "SPX_MSM_SEG1=8"])
def test_sort_form_bit_exact(setting):
    key, val = setting.split("=")
    env = dict(os.environ, **{key: val})
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "sort_form_check.py")], env=env, timeout=280,
                       capture_output=True, text=True)
    print(r.stdout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
