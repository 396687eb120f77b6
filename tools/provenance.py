"""Which code a committed profile measured: a hash of the source files themselves
(VERDICT r4 "next round" 2: evidence tagged by the sources it measured, not by a commit).

  src_sha("kernels")  — the device code: form_amd/csrc/*.hip + the device headers
                        (fmx_device.hpp, factor_rows.hpp, fmx_internal.hpp); PMC traffic
                        and SQ wave-state profiles of a kernel depend on these
  src_sha("all")      — every libfmx source (+ include/fmx): a critical-path trace also
                        depends on the host code

The GPU-side profiling tools (pmc_traffic.py, critical_path.py) stamp these into the JSON
they write, from the tree they ran; bench.py compares them with the current tree and marks
a profile whose hash differs "stale": true."""
import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_CSRC = os.path.join(ROOT, "form_amd", "csrc")
KINDS = {
    "kernels": lambda: sorted(glob.glob(os.path.join(_CSRC, "*.hip"))) +
    [os.path.join(_CSRC, f) for f in ("fmx_device.hpp", "factor_rows.hpp", "fmx_internal.hpp")],
    "all": lambda: sorted(glob.glob(os.path.join(_CSRC, "*.hip")) + glob.glob(os.path.join(_CSRC, "*.hpp")) +
                          glob.glob(os.path.join(_CSRC, "*.cpp")) + glob.glob(os.path.join(ROOT, "include", "fmx", "*"))),
}


def src_sha(kind: str = "kernels") -> str:
    h = hashlib.sha256()
    for path in KINDS[kind]():
        h.update(os.path.relpath(path, ROOT).encode())
        with open(path, "rb") as f:
            h.update(hashlib.sha256(f.read()).digest())
    return h.hexdigest()[:16]


def stamp(d: dict) -> dict:
    """Add both hashes of the current tree to a profile record."""
    d["src_sha_kernels"] = src_sha("kernels")
    d["src_sha_all"] = src_sha("all")
    return d


def staleness(d: dict, kind: str) -> dict:
    """{src_sha, stale} of a loaded profile record against the current tree (stale when it
    carries no hash: measured before hashes were recorded)."""
    have = d.get(f"src_sha_{kind}")
    return {"src_sha": have, "stale": have != src_sha(kind)}


if __name__ == "__main__":
    print(src_sha("kernels"), src_sha("all"))
