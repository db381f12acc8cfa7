"""CPU guard for the multi-process output path that turned the r4 driver suite
red: two ranks printing their JSON verdicts into one inherited stdout pipe under
PYTHONUNBUFFERED=1 produced two objects on one line.  Ranks now hand their
records to the launcher through per-rank files and every line that does reach
a shared pipe is ONE os.write (tools/jsonl.py)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import jsonl  # noqa: E402


def test_two_ranks_unbuffered_lines_never_interleave():
    lines_per_rank = 200
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rccl_loopback.py"),
                        "--n", "2", "--mode", "selftest", "--lines", str(lines_per_rank)],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    # strict: every line is exactly one object
    recs = [json.loads(x) for x in r.stdout.splitlines() if x.strip()]
    for via in ("stdout", "file"):
        for rank in (0, 1):
            got = sorted(x["i"] for x in recs if x["via"] == via and x["rank"] == rank)
            assert got == list(range(lines_per_rank)), (via, rank, len(got))
    # the merged file records come out in rank order, after both ranks exit
    merged = [x["rank"] for x in recs if x["via"] == "file"]
    assert merged == sorted(merged)


def test_records_parser_splits_concatenated_objects():
    text = ('noise\n{"a": 1}{"b": 2}\n  {"c": [1, {"d": 3}]}  \n{not json\n'
            '{"e": "}{"} {"f": 4}\n')
    assert jsonl.records(text) == [{"a": 1}, {"b": 2}, {"c": [1, {"d": 3}]}, {"e": "}{"},
                                   {"f": 4}]


def test_emit_refuses_records_longer_than_pipe_buf():
    r, w = os.pipe()
    try:
        jsonl.emit({"x": 1}, fd=w)
        assert os.read(r, 100) == b'{"x":1}\n'
        try:
            jsonl.emit({"x": "y" * 5000}, fd=w)
        except ValueError:
            pass
        else:
            raise AssertionError("oversized record was written")
    finally:
        os.close(r)
        os.close(w)
