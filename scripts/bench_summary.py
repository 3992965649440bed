"""One-screen summary of a bench.py JSON line (headline + every extra config), for GPU session logs."""
import json
import sys


def main(path):
    d = json.load(open(path))
    r = d.get("roofline") or {}
    print(f"headline {d['value']:.4g} {d['unit']}  mean {d['ms_per_step']} ms  median {d.get('ms_per_step_median')} "
          f"min {d.get('ms_per_step_min')}  busy {d.get('device_busy_ms_per_step')} ms  bitexact "
          f"{d.get('proof_bitexact_vs_cpu')}  roof {r.get('kernel')} {r.get('frac')} {r.get('avg_launch_us')}")
    for k, v in d.items():
        if not (isinstance(v, dict) and k.startswith("config")):
            continue
        if "error" in v:
            print(f"  {k}: ERROR {v['error']}")
            continue
        rr = v.get("roofline") or {}
        cpu = v.get("cpu_baseline") or {}
        print(f"  {k}: {v.get('value')} {v.get('unit')}  {v.get('ms_per_step', v.get('ms_per_prove'))} ms  "
              f"roof {rr.get('kernel')} {rr.get('frac')}  cpu {cpu.get('value') if cpu else v.get('value')}  "
              f"exact {v.get('proof_bitexact_vs_cpu', v.get('result_bitexact_vs_cpu', v.get('rows_bitexact_vs_cpu')))}")


if __name__ == "__main__":
    main(sys.argv[1])
