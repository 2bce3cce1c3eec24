"""Host sanitizer runs (CPU): the product's parser and data layer
(one-class-ffm_amd/csrc/host_data.cpp, which parses untrusted text with raw
pointers) and the oracle CLI, built with -fsanitize=address,undefined
(tests/sanitize/Makefile), over the parser's edge cases: stale label
blocks on empty lines (ffm.cpp:93), lines cut short by an unparseable token,
test features with idx >= the train Ds (ffm.cpp:104,149), CRLF, missing
values, malformed labels, empty files, huge indices, long lines, and the
chunked parallel parse.  Passing = every run ends with its documented exit
status and no sanitizer report; the chunked parses give the serial digest."""
import os
import subprocess

import numpy as np
import pytest

import synth
from test_abi_cpu import EDGE_ITEM, EDGE_TEST, EDGE_TRAIN

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(REPO, "tests", "sanitize")
DRIVER = os.path.join(SAN, "_build", "parse_driver")
ORACLE = os.path.join(SAN, "_build", "oracle_train")
ENV = dict(os.environ, ASAN_OPTIONS="abort_on_error=0:exitcode=99:detect_leaks=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=98")


@pytest.fixture(scope="module", autouse=True)
def built():
    subprocess.run(["make", "-s", "-C", SAN, "-j2"], check=True, timeout=600)


def _run(args, chunks=None, timeout=120):
    env = dict(ENV)
    if chunks is not None:
        env["OCFFM_PARSE_CHUNKS"] = str(chunks)
    r = subprocess.run(args, capture_output=True, text=True, env=env, timeout=timeout)
    for marker in ("AddressSanitizer", "LeakSanitizer", "runtime error:", "UndefinedBehaviorSanitizer"):
        assert marker not in r.stderr, r.stderr[-4000:]
    return r


def _w(tmp_path, name, text, mode="w"):
    p = tmp_path / name
    with open(p, mode) as f:
        f.write(text)
    return str(p)


def test_edge_case_files(tmp_path):
    tr, it, te = (_w(tmp_path, n, t) for n, t in (("tr", EDGE_TRAIN), ("it", EDGE_ITEM), ("te", EDGE_TEST)))
    r = _run([DRIVER, tr, it, te])
    assert r.returncode == 0, r.stdout + r.stderr
    lines = dict(line.split(" ", 1) for line in r.stdout.strip().split("\n"))
    assert "m=7 " in lines["train"] and "nnz_y=11" in lines["train"]  # the stale block counts (ffm.cpp:93)
    assert "nnz_x=2" in lines["test"]  # idx >= train Ds dropped (ffm.cpp:104,149)


ODD = {
    "empty": "",
    "blank_only": "\n\n  \t\n",
    "no_newline": "0 0:1:1 1:2:1",
    "crlf": "0,1 0:1:1\r\n1 0:2:1\r\n\r\n2 0:3:1\r\n",
    "missing_val": "0 0:1: 1:2:1\n1 0:1\n2 :1:1\n3 0::1\n",
    "garbage_tail": "0 0:1:1x 1:2:1\n1 0:1:1e400 1:1:-1e-400\n2 0:3:nan\n",
    "huge_idx": "0 0:18446744073709551615:1\n1 0:4294967296:1 1:1:1\n",
    "labels_only": "0,1,2\n3\n",
    "leading_blank": "\n\n0 0:1:1\n",
    "long_line": "0 " + " ".join(f"{i % 3}:{i}:1" for i in range(20000)) + "\n",
    "many_labels": ",".join(str(i % 7) for i in range(5000)) + " 0:1:1\n",
}


@pytest.mark.parametrize("case", sorted(ODD))
def test_odd_inputs(tmp_path, case):
    """Inputs the reference reads with undefined behaviour or its istringstream
    quirks: the product may keep or stop at them, but must stay in bounds."""
    tr = _w(tmp_path, "tr", ODD[case])
    it = _w(tmp_path, "it", EDGE_ITEM)
    te = _w(tmp_path, "te", ODD[case])
    r = _run([DRIVER, tr, it, te])
    if case == "huge_idx":  # the device layout's 32-bit indices: refused up front, not truncated
        assert r.returncode == 4 and "exceeds" in r.stdout, r.stdout + r.stderr
    else:
        assert r.returncode in (0, 3), r.stdout + r.stderr


@pytest.mark.parametrize("bad", ["1,,2 0:1:1\n", "x 0:1:1\n", ",1 0:1:1\n", "1, 0:1:1\n",
                                 "99999999999999999999999 0:1:1\n"])
def test_malformed_labels(tmp_path, bad):
    tr = _w(tmp_path, "tr", "0 0:1:1\n" + bad)
    r = _run([DRIVER, tr, _w(tmp_path, "it", EDGE_ITEM)])
    if bad.startswith("9999"):  # out_of_range from stoi, as the reference's stoi throws (uncaught there)
        assert r.returncode == 4 and "stoi" in r.stdout, r.stdout + r.stderr
    elif bad.startswith("1, "):  # a trailing comma ends the block (getline yields no empty last token)
        assert r.returncode == 0, r.stdout + r.stderr
    else:
        assert r.returncode == 3, r.stdout + r.stderr


def test_missing_file(tmp_path):
    r = _run([DRIVER, str(tmp_path / "nope"), str(tmp_path / "nope2")])
    assert r.returncode == 4


@pytest.mark.parametrize("chunks", [2, 3, 7, 16])
def test_chunked_parse(tmp_path, chunks):
    """The parallel parser (line-aligned chunks joined in file order) under
    the sanitizers, on a file with blank lines at chunk starts and lines cut
    short: the digests equal the serial parse's."""
    rng = np.random.default_rng(5)
    lines = []
    for _ in range(20000):
        r = rng.random()
        if r < 0.15:
            lines.append("" if rng.random() < 0.5 else "  \t")
            continue
        labels = ",".join(str(x) for x in rng.integers(0, 6, size=rng.integers(1, 4)))
        feats = [f"{rng.integers(0, 3)}:{rng.integers(0, 50)}:{rng.choice(['1', '0.5', '2.25e-1', '3'])}"
                 for _ in range(rng.integers(0, 5))]
        if r > 0.95:
            feats.insert(1, "junk")
        lines.append(labels + " " + " ".join(feats))
    # > 4 MB so the chunked path is taken (host_data.cpp parse_rows)
    text = "\n".join(lines) + "\n"
    text = text * (1 + (4 << 20) // len(text))
    tr = _w(tmp_path, "tr", text)
    it = _w(tmp_path, "it", EDGE_ITEM)
    serial = _run([DRIVER, tr, it], chunks=1)
    par = _run([DRIVER, tr, it], chunks=chunks)
    assert serial.returncode == 0 and par.returncode == 0, par.stdout + par.stderr
    assert par.stdout == serial.stdout


def test_oracle_cli_under_sanitizers(tmp_path):
    """The oracle (the checker every parity claim rests on) trains two epochs
    of the tiny set on 2 threads and writes its model with no sanitizer
    report."""
    ds = synth.tiny()
    paths = ds.write(str(tmp_path))
    r = _run([ORACLE, "-k", "4", "-t", "2", "-c", "2", "-p", paths["test"], "-o", str(tmp_path / "m.txt"),
              paths["item"], paths["train"]], timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert os.path.getsize(tmp_path / "m.txt") > 0
    # the stale label block and the dropped test features through the oracle's parser
    tr = _w(tmp_path, "tr", EDGE_TRAIN.replace("5,2", "5"))
    te = _w(tmp_path, "te", EDGE_TEST)
    it = _w(tmp_path, "it", EDGE_ITEM)
    r = _run([ORACLE, "-k", "4", "-t", "1", "-p", te, it, tr], timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
