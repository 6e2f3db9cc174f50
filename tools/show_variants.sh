#!/bin/bash
# summarise gpurun_out/libvar_*.json from run_variants.sh
for f in gpurun_out/libvar_*.json; do
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-1][7:-5], round(d['kernel_ms'],2), 'edge', round(d['shares']['edge'],3), 'phi_h', round(d['shares']['phi_h'],3), {k[:10]:round(v,3) for k,v in d['edge_wave0_shares_of_edge'].items()})" $f
done
