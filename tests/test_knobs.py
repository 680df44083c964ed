"""The shipped library reads only its documented runtime settings from the
environment (KODR_POOL_BYTES, KODR_HOST_THREADS, KODR_ADD_TIMING); every
other KODR_* switch goes through tune.hpp's tune_env, which reads nothing
unless the build defines KODR_TUNE (tools/ A/B builds).  Source check, CPU only."""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCUMENTED = {"KODR_POOL_BYTES", "KODR_HOST_THREADS", "KODR_ADD_TIMING"}


def test_getenv_only_for_documented_settings():
    found = set()
    for path in glob.glob(os.path.join(ROOT, "kodr_amd", "csrc", "*")):
        if not path.endswith((".cpp", ".hip", ".hpp")) or path.endswith("tune.hpp"):
            continue
        with open(path) as f:
            src = f.read()
        for m in re.finditer(r"\bgetenv\(\"([A-Z_0-9]+)\"\)", src):
            found.add(m.group(1))
        assert not re.search(r"\bgetenv\([^\"]", src), path  # no computed names
    assert found <= DOCUMENTED, found - DOCUMENTED


def test_tune_env_reads_nothing_in_the_default_build():
    with open(os.path.join(ROOT, "kodr_amd", "csrc", "tune.hpp")) as f:
        src = f.read()
    assert "#ifdef KODR_TUNE" in src and "return nullptr;" in src
    with open(os.path.join(ROOT, "kodr_amd", "build.sh")) as f:
        assert "KODR_TUNE" not in f.read().replace("KODR_TUNE_MODES", "")
