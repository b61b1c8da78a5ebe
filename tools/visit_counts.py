"""Visit counts per config from committed bench.py lines.

bench.py runs one instrumented pass outside its timed region; its exact
counters (rays, node visits and candidate tests per ray, per bounce, for
extension and shadow rays) are deterministic given the seed.  This tool
copies them out of a bench line into `profiles/visit_counts_<config>.json`
together with SURVEY §8(d)'s algorithmic bytes per sample, so that the
roofline figure can be recomputed from the committed numbers alone:

  extension ray  28 B + 32 B per node + 32 B per candidate + 16 B hit
  shadow ray     28 B + 32 B per node + 32 B per candidate + 4 B result
  (bench.py's k_extend `bytes_per_launch` is the extension-ray sum.)

usage: python tools/visit_counts.py profiles/r02w_bench.json [more lines ...]
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def last_line(path):
    return json.loads(open(path).read().strip().splitlines()[-1])


def counts(d):
    f = d["frame"]
    cfg = d["config"]
    samples = cfg["width"] * cfg["height"] * cfg["spp"]
    ext_b = sh_b = 0.0
    rows = []
    for b in f["per_bounce"]:
        n_e, n_s = b["rays"], b.get("shadow_rays", 0)
        e = n_e * (28 + 16 + 32 * (b["nodes_per_ray"] + b["prims_per_ray"]))
        s = n_s * (28 + 4 + 32 * (b.get("shadow_nodes_per_ray", 0.0) + b.get("shadow_prims_per_ray", 0.0)))
        ext_b += e
        sh_b += s
        rows.append({k: b[k] for k in ("bounce", "rays", "nodes_per_ray", "prims_per_ray", "shadow_rays",
                                       "shadow_nodes_per_ray", "shadow_prims_per_ray") if k in b})
    return {
        "config": cfg.get("config"),
        "workload": cfg.get("workload"),
        "samples_per_frame": samples,
        "per_bounce": rows,
        "extension_bytes_per_frame": round(ext_b),
        "shadow_bytes_per_frame": round(sh_b),
        "extension_bytes_per_sample": round(ext_b / samples, 1),
        "shadow_bytes_per_sample": round(sh_b / samples, 1),
        "source_line": {"value": d["value"], "unit": d["unit"], "ms_per_step": d["ms_per_step"],
                        "roofline_frac": d["roofline"]["frac"]},
        "note": "per-ray figures are rounded to 2 decimals in the bench line, so recomputed bytes agree with "
                "bench.py's exact-count bytes_per_launch to ~1e-4",
    }


def main(paths):
    for p in paths:
        d = last_line(p)
        out = counts(d)
        name = str(out["config"])
        dst = os.path.join(HERE, "..", "profiles", f"visit_counts_{name}.json")
        out["source"] = os.path.basename(p)
        with open(dst, "w") as fh:
            json.dump(out, fh, indent=1)
            fh.write("\n")
        print(f"{dst}: {out['extension_bytes_per_sample']} B/sample extension, "
              f"{out['shadow_bytes_per_sample']} B/sample shadow")


if __name__ == "__main__":
    main(sys.argv[1:])
