"""Check that the in-tree libccsc.so was linked from the sources in this tree: build.py
writes the hash of every source and header it compiled next to the library
(libccsc.srchash); this recomputes it.  The suite scripts (gpu_suite.sh, gpu_final.sh) run
it first, so committed GPU evidence cannot come from a leftover A/B variant.
Exit status 0 = current, 1 = stale or missing."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from ccsc_code_iccv2017_amd import build  # noqa: E402

want = build.source_hash()
stamp = build.LIB.with_suffix(".srchash")
got = stamp.read_text().strip() if stamp.exists() else "missing"
if got != want:
    print(f"libccsc.so is not the build of this tree (stamp {got[:16]}, sources {want[:16]}): "
          "run python -m ccsc_code_iccv2017_amd.build", file=sys.stderr)
    sys.exit(1)
print(f"libccsc.so current (sources {want[:16]})")
