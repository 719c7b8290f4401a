#!/bin/bash
# one line per variant of a tools/small_n_ab.sh output directory
for f in "$1"/*.json; do
  i=${f%.json}
  python3 -c "
import json,sys
d=json.load(open('$f')); k=d['kernels']
print('%-40s %7.1f M/s  ms %.4f  comb %.4f  scal %.4f  %s' % (open('$i.variant').read().strip(), d['value']/1e6, d['ms_per_step'], k['ecdsa_comb']['avg_ms'], k['ecdsa_scalars']['avg_ms'], d['check']))"
done
