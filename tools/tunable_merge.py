#!/usr/bin/env python
"""Merge the result lines of a TunableOp tuning run into the shipped table
(datamining_recblr_amd/tuning/gemm_gfx950.csv): the validator lines must
agree; result lines of the new file replace same-key lines of the old.

    python tools/tunable_merge.py <new.csv> [table.csv]"""
import sys


def read(p):
    val, res = {}, {}
    for line in open(p):
        parts = line.rstrip("\n").split(",")
        if len(parts) < 3:
            continue
        if parts[0] == "Validator":
            val[parts[1]] = ",".join(parts[2:])
        else:
            res[(parts[0], parts[1])] = line.rstrip("\n")
    return val, res


def main():
    new = sys.argv[1]
    table = sys.argv[2] if len(sys.argv) > 2 else "datamining_recblr_amd/tuning/gemm_gfx950.csv"
    v0, r0 = read(table)
    v1, r1 = read(new)
    for k in v0:
        if k in v1 and v1[k] != v0[k]:
            raise SystemExit(f"validator {k} differs: {v0[k]} vs {v1[k]}")
    added = [k for k in r1 if k not in r0]
    r0.update(r1)
    with open(table, "w") as f:
        for k, v in v0.items():
            f.write(f"Validator,{k},{v}\n")
        for line in r0.values():
            f.write(line + "\n")
    print(f"merged {len(r1)} results ({len(added)} new) into {table}")
    for k in added:
        print("  +", r1[k][:140])


if __name__ == "__main__":
    main()
