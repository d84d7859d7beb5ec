"""Print chosen keys of the last JSON line of a file (bench / probe output that
may carry library banners before it).  usage: last_json.py FILE KEY..."""
import json
import sys

d = json.loads([ln for ln in open(sys.argv[1]) if ln.startswith("{")][-1])
print(json.dumps({k: d.get(k) for k in sys.argv[2:]}))
