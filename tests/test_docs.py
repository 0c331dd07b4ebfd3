"""The docs name only things that exist (docs/PARITY.md still listed deleted
knobs and a deleted test). Checked on every ``tests/*.py`` path, ``file.py::test_name`` reference,
``MBK_*`` switch and ``--flag`` that docs/PARITY.md and README.md mention."""
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
DOCS = [ROOT / "docs" / "PARITY.md", ROOT / "README.md"]


def _text():
    return {p.name: p.read_text() for p in DOCS}


def test_named_test_files_and_functions_exist():
    for name, text in _text().items():
        for path in set(re.findall(r"(tests/[\w/]+\.py)", text)):
            assert (ROOT / path).exists(), f"{name} names missing {path}"
        for path, fn in set(re.findall(r"(tests/[\w/]+\.py)::(\w+)", text)):
            src = (ROOT / path).read_text()
            assert re.search(rf"^def {fn}\(", src, re.M), f"{name} names missing {path}::{fn}"


def test_named_env_switches_exist():
    from test_knobs import KNOBS
    for name, text in _text().items():
        for k in set(re.findall(r"\b(MBK_[A-Z0-9_]+)", text)):
            assert k in KNOBS, f"{name} names {k}, which is not a documented switch"


def test_named_flags_exist():
    """Every ``--flag`` in backticks is a flag of the training CLI, bench.py or a tools/ script."""
    srcs = [ROOT / "microbeast_amd" / "config.py", ROOT / "bench.py"]
    srcs += sorted((ROOT / "tools").glob("*.py")) + sorted((ROOT / "tools").glob("*.sh"))
    import dataclasses

    from microbeast_amd.config import Flags
    known = {"--" + f.name for f in dataclasses.fields(Flags)}  # config.py: a flag per field
    for p in srcs:
        known |= set(re.findall(r"""["'](--[a-z0-9_]+)["']""", p.read_text()))
        known |= set(re.findall(r"(--[a-z0-9_]+)", p.read_text())) if p.suffix == ".sh" else set()
    for name, text in _text().items():
        for code in re.findall(r"`([^`]*)`", text):
            for f in re.findall(r"(?<![\w-])(--[a-z][a-z0-9_]+)(?![\w-])", code):
                assert f in known, f"{name} names flag {f}, which no parser defines"
