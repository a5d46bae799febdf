import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def record_parity(test: str, **values):
    """Append measured parity numbers of a GPU test to $OSPO_PARITY_LOG (JSON lines), so the
    tolerances written in the tests can be checked against what was measured."""
    path = os.environ.get("OSPO_PARITY_LOG")
    if not path:
        return
    import json
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "a") as f:
        f.write(json.dumps({"test": test, **{k: (float(v) if not isinstance(v, (str, list, dict)) else v)
                                             for k, v in values.items()}}) + "\n")
