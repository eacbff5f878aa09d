"""Run sizes in a server request trace (PS_TRACE_REQUESTS lines: server sender
ts push pull keys run_size run_pos): per server, how many requests were taken
alone and how many in runs of each size, split by request kind."""
import collections
import sys

runs = collections.defaultdict(collections.Counter)
kinds = collections.defaultdict(collections.Counter)
for line in open(sys.argv[1]):
    f = line.split()
    if len(f) != 8:
        continue
    server, push, pull, rs, rp = int(f[0]), int(f[3]), int(f[4]), int(f[6]), int(f[7])
    if rp == 0:
        runs[server][rs] += 1
    kinds[server][("push" if push else "") + ("pull" if pull else "") + f"@{rs}"] += 1
for s in sorted(runs):
    print(f"server {s}: runs by size {dict(sorted(runs[s].items()))}; requests {dict(sorted(kinds[s].items()))}")
