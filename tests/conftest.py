import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tools"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libcloudsc_amd.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def ds():
    import cloudsc_amd as ca
    return ca.load_dataset()


@pytest.fixture(scope="session")
def scenarios(ds):
    import make_fixtures as mf
    return {name: mf.load_scenario(name, ds) for name in ("W", "M")}


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    if not os.path.exists(oracle.ORACLE_LIB):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle"), "liboracle.so"])
    return oracle
