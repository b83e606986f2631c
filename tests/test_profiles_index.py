"""profiles/README.md indexes every evidence file under profiles/ (VERDICT r05 "stop the
evidence sprawl"): each tracked file is named there, by its path relative to profiles/, its
file name, or a glob (`r05at_*`, `r05ap_prof_{c1,c2}.md`).  CPU only."""
import fnmatch
import os
import re
import subprocess

from tests.conftest import ROOT


def _globs(text):
    out = []
    for tok in re.findall(r"`([^`]+)`", text):
        for part in tok.split():
            m = re.match(r"(.*)\{([^}]*)\}(.*)", part)
            if m:
                out += [m.group(1) + alt + m.group(3) for alt in m.group(2).split(",")]
            elif part:
                out.append(part)
    return out


def test_every_profile_file_is_indexed():
    try:
        files = subprocess.check_output(["git", "ls-files", "profiles"], cwd=ROOT, text=True).split()
    except (OSError, subprocess.CalledProcessError):
        files = [os.path.relpath(os.path.join(d, f), ROOT) for d, _, fs in os.walk(os.path.join(ROOT, "profiles"))
                 for f in fs]
    text = open(os.path.join(ROOT, "profiles", "README.md")).read()
    pats = _globs(text)
    missing = []
    for f in files:
        rel = os.path.relpath(f, "profiles")
        if rel == "README.md":
            continue
        names = {rel, os.path.basename(rel), "profiles/" + rel}
        if not any(fnmatch.fnmatch(n, p) for n in names for p in pats):
            missing.append(rel)
    assert not missing, f"{len(missing)} profile files not listed in profiles/README.md, e.g. {missing[:10]}"
