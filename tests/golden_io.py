"""Load tests/golden/cases.json (fixtures only: inputs + expected outputs)."""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def dec(d) -> bytes:
    if "hex" in d:
        return bytes.fromhex(d["hex"])
    return b"".join(bytes.fromhex(h) * n for h, n in d["rle"])


def load_cases(kind=None):
    with open(os.path.join(HERE, "golden", "cases.json")) as f:
        cases = json.load(f)["cases"]
    return [c for c in cases if kind is None or c["kind"] == kind]
