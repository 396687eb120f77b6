"""Tag committed profile JSON files with the commit of the code they measured.

  python tools/tag_profile.py <commit-ish> profiles/traffic_latest.json [...]

Adds "measured_at": <full hash of commit-ish> (the code that ran on the GPU box; the
profile itself is committed afterwards), so bench.py's roofline block can say which
build its PMC traffic and SQ wave-state figures come from."""
import json
import subprocess
import sys


def main():
    rev = subprocess.check_output(["git", "rev-parse", sys.argv[1]], text=True).strip()
    for path in sys.argv[2:]:
        with open(path) as f:
            d = json.load(f)
        d["measured_at"] = rev
        with open(path, "w") as f:
            json.dump(d, f, indent=1)
        print(path, rev[:12])


if __name__ == "__main__":
    main()
