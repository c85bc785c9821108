"""Every ``<file>:<line>`` citation in this repository points at lines that exist.

Reference citations (FEDn v0.33.0, ``/root/reference``; skipped when the checkout is absent, e.g.
on the GPU box) are resolved by path suffix — ``fedn/network/combiner/aggregators/fedavg.py:47-50``
or the bare ``fedavg.py:47-50`` — and must be in range for the cited file (for a bare name that
several reference files share, for at least one of them). Citations of this repository's own
files (``fedn_amd/…``, ``tests/…``, ``tools/…``, ``oracle/…``, ``include/…``, ``bench.py``) are
checked against the repository. Lists (``fedavg.py:37-39, 80``) are checked number by number.

The judge's documents (SURVEY/VERDICT/ADVICE/BASELINE/PAPERS/SNIPPETS.md) are not ours to edit and
are not scanned; nor are test fixtures and run outputs.
"""
import collections
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
REPO_PREFIXES = ("fedn_amd/", "tests/", "tools/", "oracle/", "include/")
REPO_FILES = ("bench.py", "__graft_entry__.py")
NOT_OURS = {"SURVEY.md", "VERDICT.md", "ADVICE.md", "PAPERS.md", "SNIPPETS.md", "BASELINE.md"}
SKIP_DIRS = {".git", "gpurun_out", "__pycache__", "golden", ".pytest_cache", "profiles"}
CITE = re.compile(r"(?<![\w/.-])([\w./-]+\.(?:py|proto|rst|yaml|toml|sh|ipynb|hip|h|cpp|c))"
                  r"(:\d+(?:-\d+)?(?:, ?\d+(?:-\d+)?)*)")


def _sources():
    for dp, dns, fns in os.walk(ROOT):
        dns[:] = [d for d in dns if d not in SKIP_DIRS]
        for f in fns:
            if f.endswith((".py", ".md", ".h", ".hip", ".cpp", ".c")) and f not in NOT_OURS:
                yield os.path.join(dp, f)


def _citations():
    for path in _sources():
        with open(path, errors="replace") as fh:
            for ln, line in enumerate(fh, 1):
                for m in CITE.finditer(line):
                    yield os.path.relpath(path, ROOT), ln, m.group(1), [int(x) for x in re.findall(r"\d+", m.group(2))]


_lines = {}


def _nlines(path):
    if path not in _lines:
        with open(path, "rb") as fh:
            _lines[path] = sum(1 for _ in fh)
    return _lines[path]


def _is_repo(name):
    return name.startswith(REPO_PREFIXES) or name in REPO_FILES


def test_repo_citations_in_range():
    bad = []
    for src, ln, name, nums in _citations():
        if not _is_repo(name):
            continue
        target = os.path.join(ROOT, name)
        if not os.path.exists(target):
            continue                        # e.g. a path relative to another package; not resolvable
        n = _nlines(target)
        if any(x < 1 or x > n for x in nums):
            bad.append(f"{src}:{ln}: {name}:{nums} (file has {n} lines)")
    assert not bad, "out-of-range citations of repository files:\n" + "\n".join(bad)


@pytest.mark.skipif(not os.path.isdir(REF), reason="the FEDn reference checkout is only in the build container")
def test_reference_citations_in_range():
    by_name = collections.defaultdict(list)
    for dp, dns, fns in os.walk(REF):
        dns[:] = [d for d in dns if d != ".git"]
        for f in fns:
            by_name[f].append(os.path.relpath(os.path.join(dp, f), REF))
    bad, checked = [], 0
    for src, ln, name, nums in _citations():
        if _is_repo(name):
            continue
        base = os.path.basename(name)
        cands = by_name.get(base, [])
        if "/" in name:
            cands = [c for c in cands if ("/" + c).endswith("/" + name.lstrip("./"))]
        if not cands:
            continue                        # not a reference file (one of ours cited by bare name, …)
        checked += 1
        if not any(all(1 <= x <= _nlines(os.path.join(REF, c)) for x in nums) for c in cands):
            bad.append(f"{src}:{ln}: {name}:{nums} (candidates: "
                       + ", ".join(f"{c} has {_nlines(os.path.join(REF, c))} lines" for c in cands) + ")")
    assert checked > 300, f"only {checked} reference citations found: the scanner is broken"
    assert not bad, f"{len(bad)} out-of-range reference citations:\n" + "\n".join(bad)
