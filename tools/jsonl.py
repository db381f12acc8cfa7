"""One-record-per-line JSON output that survives several processes sharing a pipe.

`print(json.dumps(x), flush=True)` may reach the pipe as two writes (the text,
then the newline) when stdout is unbuffered (PYTHONUNBUFFERED=1), and another
process's line can land between them: two objects on one line (the r4 driver
suite failed on exactly that, tools/rccl_loopback.py --mode developed).
`emit` issues the whole line, newline included, as ONE os.write; a pipe write
of at most PIPE_BUF (4096) bytes is atomic, and longer records are refused
rather than risked.  `records` parses a captured stream tolerantly: every JSON
object that starts a line, several per line if a writer elsewhere still
concatenates them.
"""
import json
import os

PIPE_BUF = 4096


def emit(obj, fd=1):
    data = (json.dumps(obj, separators=(",", ":")) + "\n").encode()
    if len(data) > PIPE_BUF:
        raise ValueError(f"record of {len(data)} bytes exceeds PIPE_BUF ({PIPE_BUF}); "
                         "write it to a per-rank file instead")
    n = os.write(fd, data)
    if n != len(data):
        raise OSError(f"short write: {n} of {len(data)} bytes")


def append_record(path, obj):
    """Append one record to a per-rank result file (one writer per file)."""
    with open(path, "a") as f:
        f.write(json.dumps(obj, separators=(",", ":")) + "\n")


def read_records(path):
    if not os.path.exists(path):
        return []
    with open(path) as f:
        return [json.loads(x) for x in f.read().splitlines() if x.strip()]


def records(text):
    """Every JSON object that begins a line of `text`, including objects
    concatenated onto the same line."""
    dec = json.JSONDecoder()
    out = []
    for line in text.splitlines():
        s = line.strip()
        i = 0
        while i < len(s) and s[i] == "{":
            try:
                obj, end = dec.raw_decode(s, i)
            except ValueError:
                break   # a log line that merely starts with '{'
            out.append(obj)
            i = end
            while i < len(s) and s[i].isspace():
                i += 1
    return out
