"""Documentation stays in step with the code: every PYRECOVER_* / PRA_* environment knob the framework
reads (Python package, native sources, bench.py / train.py) is listed in docs/KNOBS.md."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PREFIXES = {"PYRECOVER_ATTN_", "PYRECOVER_RCCL_", "PYRECOVER_RCCL"}  # prefixes of documented families


def _sources():
    for base in ("pyrecover_amd", "csrc"):
        for dirpath, _, files in os.walk(os.path.join(ROOT, base)):
            for f in files:
                if f.endswith((".py", ".h", ".cpp", ".hip")):
                    yield os.path.join(dirpath, f)
    for f in ("bench.py", "train.py"):
        yield os.path.join(ROOT, f)


def test_every_environment_knob_is_documented():
    names = set()
    for path in _sources():
        with open(path, encoding="utf-8", errors="replace") as fh:
            text = fh.read()
        names.update(re.findall(r"PYRECOVER_[A-Z0-9_]+", text))
        # PRA_* names are also compile-time macros; only the ones read from the environment count
        names.update(re.findall(r"(?:environ\.get|getenv)\(\s*[\"'](PRA_[A-Z0-9_]+)", text))
    names -= PREFIXES
    with open(os.path.join(ROOT, "docs", "KNOBS.md"), encoding="utf-8") as fh:
        doc = fh.read()
    documented = set(re.findall(r"(?:PYRECOVER|PRA)_[A-Z0-9_]+", doc))
    # "PYRECOVER_ATTN_FWD_ORDER`, `_DQ_ORDER`" style rows document a family member by suffix
    documented |= {"PYRECOVER_ATTN" + m for m in re.findall(r"`(_[A-Z0-9_]+)`", doc)}
    attn_keys = {"PYRECOVER_ATTN_" + k.upper() for k in __import__("pyrecover_amd._ext", fromlist=["x"])._ATTN_ENV}
    missing = sorted((names | attn_keys) - documented)
    assert not missing, f"undocumented knobs (add them to docs/KNOBS.md): {missing}"


def test_user_knobs_at_most_thirty():
    """docs/KNOBS.md: at most 30 user-facing knobs (the test and fault-injection hooks are listed
    separately), and every documented knob is still read by the code."""
    import re as _re

    with open(os.path.join(ROOT, "docs", "KNOBS.md"), encoding="utf-8") as fh:
        doc = fh.read()
    user, _, hooks = doc.partition("## Test and fault-injection hooks")
    user_names = set(_re.findall(r"(?:PYRECOVER|PRA)_[A-Z0-9_]+", user.split("## Kernels and schedules", 1)[1]))
    assert len(user_names) <= 30, sorted(user_names)
    read = set()
    for path in _sources():
        with open(path, encoding="utf-8", errors="replace") as fh:
            read.update(_re.findall(r"(?:PYRECOVER|PRA)_[A-Z0-9_]+", fh.read()))
    stale = sorted(n for n in user_names | set(_re.findall(r"(?:PYRECOVER|PRA)_[A-Z0-9_]+", hooks)) if n not in read)
    assert not stale, f"documented but never read: {stale}"
