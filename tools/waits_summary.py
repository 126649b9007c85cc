#!/usr/bin/env python3
"""Summarise one rocprofv3 --pmc pass of SQ wait/active counters over the
one-tick step kernel's launches (tools/gpu_r3*.sh):
    python tools/waits_summary.py <run dir> <workload>  ->  <run dir>/waits_<wl>.json
SQ_WAVE_CYCLES ~= SQ_WAIT_ANY (parked on s_waitcnt / barrier / s_sleep) +
SQ_WAIT_INST_ANY (ready but stalled at issue) + SQ_ACTIVE_INST_ANY (issuing),
all in quad-cycles summed over the launch's waves (MI355X_MICROARCH.md)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import counters  # noqa: E402


def main():
    out, wl = sys.argv[1], sys.argv[2]
    c, n = counters(os.path.join(out, 'run_counter_collection.csv'))
    g = lambda k: next((v for name, v in c.items() if name == k or name == k + '_sum'), 0.0)  # noqa: E731
    wc = g('SQ_WAVE_CYCLES')
    res = dict(workload=wl, launches=max(n.values()) if n else 0, per_launch={k: v for k, v in sorted(c.items())},
               frac_of_wave_cycles=dict(wait_any=g('SQ_WAIT_ANY') / wc, wait_inst_any=g('SQ_WAIT_INST_ANY') / wc,
                                        active_inst_any=g('SQ_ACTIVE_INST_ANY') / wc,
                                        active_valu=g('SQ_ACTIVE_INST_VALU') / wc,
                                        active_lds=g('SQ_ACTIVE_INST_LDS') / wc),
               lds_bank_conflict_per_lds_active=g('SQ_LDS_BANK_CONFLICT') / max(g('SQ_ACTIVE_INST_LDS'), 1.0),
               note='quad-cycles summed over the launch waves (step and helper waves together), averaged over '
                    'the one-tick step kernel launches after the first 10')
    json.dump(res, open(os.path.join(out, 'waits_%s.json' % wl), 'w'), indent=1)
    print(json.dumps(res['frac_of_wave_cycles']), res['lds_bank_conflict_per_lds_active'])


if __name__ == '__main__':
    main()
