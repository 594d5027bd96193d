"""Test configuration. `-m gpu` tests run the HIP library on an MI355X and compare it with the
oracle (oracle/: CPU restatements = test infrastructure only); `-m "not gpu"` tests cover the
oracle against the reference invariants / golden fixtures, the host logic, and that the C-ABI
library loads and exports every symbol of include/spartan_hip.h."""
import importlib.util
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle", "py"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library)")
    config.addinivalue_line("markers", "slow: longer CPU-only cases")
    hb = os.environ.get("SPX_HEARTBEAT")
    if hb:
        # long single tests (the oracle proving 2^22 for ~2 min) print nothing meanwhile: a line every
        # 20 s into this file shows a remote runner that the run is alive
        import threading
        import time

        def beat():
            t0 = time.time()
            while True:
                with open(hb, "a") as f:
                    f.write("alive %.0f s\n" % (time.time() - t0))
                time.sleep(20)

        threading.Thread(target=beat, daemon=True).start()


def load_product():
    spec = importlib.util.spec_from_file_location("r1cs_spartan_amd", os.path.join(ROOT, "r1cs-spartan_amd", "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["r1cs_spartan_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def ensure_oracle_lib():
    so = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(so):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    return so


@pytest.fixture(scope="session")
def oc():
    ensure_oracle_lib()
    import oracle_c

    return oracle_c


@pytest.fixture(scope="session")
def spx():
    return load_product()


@pytest.fixture(scope="session")
def ctx(spx):
    return spx.Context(0)
