"""Both forms of the hand-written MSM bucket sort (msm_common.hip: the LDS-staged form chosen for
dense batches, the direct form for a sharded rank's sparse ones), each forced for a whole child
process by SPX_SORT_FORM, against the oracle byte for byte (tests/sort_form_check.py)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("form", ["staged", "direct"])
def test_sort_form_bit_exact(form):
    env = dict(os.environ, SPX_SORT_FORM=form)
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "sort_form_check.py")], env=env, timeout=280,
                       capture_output=True, text=True)
    print(r.stdout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
