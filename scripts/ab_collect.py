#!/usr/bin/env python3
"""Collect tune_b3.py A/B outputs from several GPU-box calls into one JSONL
under profiles/ (one header line, then every variant row tagged with its call).
usage: scripts/ab_collect.py OUT.jsonl NOTE  TAG:FILE:VARIANTS ..."""
import json
import sys


def main():
    out, note, specs = sys.argv[1], sys.argv[2], sys.argv[3:]
    with open(out, "w") as o:
        o.write(json.dumps({"note": note}) + "\n")
        for spec in specs:
            tag, path, variants = spec.split(":", 2)
            for line in open(path):
                line = line.strip()
                if not line.startswith("{"):
                    continue
                d = json.loads(line)
                d["box_call"] = tag
                d["variants"] = variants
                o.write(json.dumps(d) + "\n")


if __name__ == "__main__":
    main()
