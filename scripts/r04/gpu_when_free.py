"""Runs one gpurun command when the pool lets it start: a call that ended
with status "transient" (no box, back-off, box lost while being prepared:
nothing of the command ran, nothing charged) is tried again after the wait
gpurun names; any other outcome (ok, fail, timeout) is final.
    python3 scripts/r04/gpu_when_free.py OUTFILE TIMEOUT 'command'"""
import json
import re
import subprocess
import sys
import time

out, timeout, cmd = sys.argv[1], sys.argv[2], sys.argv[3]
for attempt in range(12):
    with open(out, "w") as f:
        subprocess.run(["/usr/local/graft/bin/gpurun", "--timeout", timeout, "--", cmd], stdout=f,
                       stderr=subprocess.STDOUT)
    text = open(out).read()
    try:
        status = json.load(open("gpurun_out/.last_call.json")).get("status")
    except Exception:
        status = None
    if "status=transient" not in text:
        break
    m = re.search(r"retry in (\d+)s", text)
    wait = int(m.group(1)) + 10 if m else 150
    print(f"attempt {attempt}: transient ({status}), waiting {wait} s", flush=True)
    time.sleep(wait)
print(text[-4000:])
