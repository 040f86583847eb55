#!/usr/bin/env python3
"""Summary of the full-grid parity reports (tests/test_gpu_config34.py, test_gpu_parity.py::
test_large_grid_full, written to gpurun_out/parity/): per workload, variant and field the
cells compared, the cells over 1e-10 by the mixed gate and by plain relative
error, the worst of each, and how far the cells over the gate are inside their conditioning
allowance (error / twice the oracle's movement under 16-ulp input perturbations).

  python parity_summary.py <reports dir> > summary.json
"""
import glob
import json
import os
import sys


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/parity"
    out, totals = {}, {"cell_values": 0, "cells_mixed_gt_1e-10": 0, "cells_rel_gt_1e-10": 0, "worst_err_over_movement": 0.0}
    for f in sorted(glob.glob(os.path.join(d, "*.json"))):
        name = os.path.basename(f)[:-5]
        if name == "summary":
            continue
        rep = json.load(open(f))
        groups = [(name, rep)] if any(k.count(":") == 2 for k in rep) else [(f"{name} {k}", v) for k, v in rep.items()]
        for label, fields in groups:
            # variants: 'config3 CCLM', shards folded into the variant
            key = label.split(" shard ")[0]
            row = out.setdefault(key, {})
            for fk, v in fields.items():
                r = row.setdefault(fk, {"cells": 0, "cells_mixed_gt_1e-10": 0, "cells_rel_gt_1e-10": 0, "max_mixed": 0.0,
                                        "max_rel": 0.0, "bit_identical_cells": 0, "worst_err_over_movement": 0.0})
                r["cells"] += v["cells"]
                r["cells_mixed_gt_1e-10"] += v["cells_mixed_gt_1e-10"]
                r["cells_rel_gt_1e-10"] += v["cells_rel_gt_1e-10"]
                r["max_mixed"] = max(r["max_mixed"], v["mixed"])
                r["max_rel"] = max(r["max_rel"], v["max_rel"])
                r["bit_identical_cells"] += v["bit_identical_cells"]
                c = v.get("conditioned", {}).get("max_err_over_movement", 0.0)
                r["worst_err_over_movement"] = max(r["worst_err_over_movement"], c)
                totals["cell_values"] += v["cells"]
                totals["cells_mixed_gt_1e-10"] += v["cells_mixed_gt_1e-10"]
                totals["cells_rel_gt_1e-10"] += v["cells_rel_gt_1e-10"]
                totals["worst_err_over_movement"] = max(totals["worst_err_over_movement"], c)
    print(json.dumps({"totals": totals, "by_workload": out,
                      "rule": "cells_mixed_gt_1e-10: over the SURVEY 8d gate |x - ref| / max(|ref|, 1e-6 |ref|_inf); "
                              "each such cell must be within twice the oracle's own movement under 16-ulp input "
                              "perturbations (tests/parity.py::conditioned_full): worst_err_over_movement is the "
                              "largest error / (that movement) seen, the allowance being 2"}, indent=1))


if __name__ == "__main__":
    main()
