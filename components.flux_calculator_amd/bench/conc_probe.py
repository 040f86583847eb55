import json, sys, types
sys.path.insert(0, '.')
sys.path.insert(0, 'components.flux_calculator_amd/python')
import bench
a = types.SimpleNamespace(types=1, bias=False)
v = ("CCLM", "MOM5", "RCO")
seq = bench.e2e_host(a, v, sizes=(32_768,))
conc = bench.e2e_concurrent(a, v)
conc2 = bench.e2e_concurrent(a, v)
print(json.dumps({"seq": seq["sizes"]["32768"], "conc": conc, "conc2": conc2}))
