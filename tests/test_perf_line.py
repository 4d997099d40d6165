"""The GPU tier's PERF summary line: tests/conftest.py
prints the perf floors' in-memory records as one line right above pytest's
final "N passed" line, whether the floors pass or fail -- the only part of a
passing GPU tier's output the driver keeps is its tail."""
import os
import shutil

pytest_plugins = ["pytester"]

HERE = os.path.dirname(os.path.abspath(__file__))

RECORDING_TEST = '''
from conftest import PERF_RECORDS


def test_records():
    PERF_RECORDS.update(fill=6.93125, verify_lds8=5.8, rccl=1233.5)


def test_floor():
    assert PERF_RECORDS["fill"] > {floor}
'''


def _run(pytester, floor):
    shutil.copy(os.path.join(HERE, "conftest.py"), pytester.path / "conftest.py")
    pytester.makepyfile(test_rec=RECORDING_TEST.format(floor=floor))
    return pytester.runpytest_subprocess("-q", "-p", "no:cacheprovider")


def test_perf_line_sits_above_the_final_summary(pytester):
    res = _run(pytester, 5.5)
    lines = [l for l in res.outlines if l.strip()]
    assert lines[-1].startswith("2 passed"), res.outlines
    assert lines[-2] == "PERF fill=6.931 verify_lds8=5.8 rccl=1234", res.outlines


def test_perf_line_is_printed_when_a_floor_fails(pytester):
    res = _run(pytester, 7.5)
    assert res.ret != 0
    perf = [l for l in res.outlines if l.startswith("PERF ")]
    assert perf == ["PERF fill=6.931 verify_lds8=5.8 rccl=1234"], res.outlines
    assert "1 failed, 1 passed" in res.outlines[-1]


def test_no_perf_line_without_records(pytester):
    shutil.copy(os.path.join(HERE, "conftest.py"), pytester.path / "conftest.py")
    pytester.makepyfile(test_plain="def test_x():\n    pass\n")
    res = pytester.runpytest_subprocess("-q", "-p", "no:cacheprovider")
    assert res.ret == 0 and not [l for l in res.outlines if l.startswith("PERF")]
