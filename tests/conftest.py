import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O


def rfc_input(entry):
    if "input_hex" in entry:
        return bytes.fromhex(entry["input_hex"])
    return {"zeros32": bytes(32), "ff32": b"\xff" * 32, "inc32": bytes(range(32)),
            "dec32": bytes(range(31, -1, -1))}[entry["input"]]


def copyset_files(g):
    return {k: (bytes(g["copyset_hash"]["zero_file_bytes"]) if v is None else v.encode())
            for k, v in g["copyset_hash"]["files"].items()}
