"""Print one line per bench JSON: value, us/step, roofline frac (tools helper)."""
import json
import sys

for f in sys.argv[1:]:
    try:
        j = json.load(open(f))
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable:", e)
        continue
    r = j.get("roofline", {})
    print(f"{f}: {j['value'] / 1e9:.3f} G/s  {j['ms_per_step'] * 1e3:.1f} us/step  "
          f"kernel {r.get('kernel_ms', 0) * 1e3:.1f} us  frac {r.get('frac', 0):.4f}  traffic {r.get('traffic')}")
