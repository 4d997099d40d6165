"""docs/ENVIRONMENT.md lists every P2P_* variable the framework reads.

The names are collected from the sources: the native engine's getenv /
env_int / setenv calls, the Python package's and bench.py's os.environ reads,
and the test / script helpers.  A knob added without a line in the page fails
here.
"""

import os
import re

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
DOC = os.path.join(ROOT, "docs", "ENVIRONMENT.md")

# A P2P_* name in a string literal.  P2P_RCCL_PREV_ + a name is listed as
# P2P_RCCL_PREV_<name>; other literals ending in "_" are prefixes.
_NAME = re.compile(r"[\"'](P2P_[A-Z0-9_]+)")
_SOURCES = (
    ("csrc", (".cpp", ".hpp", ".hip")),
    ("test_nccl_p2p_amd", (".py",)),
    ("tests", (".py",)),
    ("scripts", (".py", ".sh")),
)
# Literals that are not variables the framework reads.
_NOT_VARIABLES = {"P2P_TEST_DATA"}  # a compile-time macro of the host tests (Makefile)


def _names():
    found = {}
    files = [os.path.join(ROOT, "bench.py")]
    for top, exts in _SOURCES:
        for d, dirs, fs in os.walk(os.path.join(ROOT, top)):
            dirs[:] = [x for x in dirs if x not in ("probes", "__pycache__", "data")]
            files += [os.path.join(d, f) for f in fs if f.endswith(exts)]
    for path in files:
        if os.path.abspath(path) == os.path.abspath(__file__):
            continue
        with open(path, errors="replace") as f:
            for m in _NAME.finditer(f.read()):
                found.setdefault(m.group(1), os.path.relpath(path, ROOT))
    return found


def test_every_p2p_variable_is_documented():
    with open(DOC) as f:
        doc = f.read()
    names = _names()
    assert len(names) > 30, sorted(names)
    missing = []
    for name, where in sorted(names.items()):
        if name in _NOT_VARIABLES:
            continue
        if name.startswith("P2P_RCCL_PREV_"):
            name = "P2P_RCCL_PREV_<name>"
        elif name.endswith("_"):  # a prefix the code matches names against
            if "`" + name not in doc:
                missing.append("%s* (%s)" % (name, where))
            continue
        if not re.search("`" + re.escape(name) + "[`=]", doc):
            missing.append("%s (%s)" % (name, where))
    assert not missing, "add these to docs/ENVIRONMENT.md: " + ", ".join(missing)


def test_documented_variables_exist():
    # The page lists no variable that nothing reads any more.
    with open(DOC) as f:
        listed = set(re.findall(r"`(P2P_[A-Z0-9_]+)", f.read()))
    names = set(_names())
    stale = sorted(x for x in listed if x not in names and x.rstrip("_") + "_" not in names)
    assert not stale, "docs/ENVIRONMENT.md lists variables nothing reads: %s" % stale
