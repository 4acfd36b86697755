"""CPU restatement of the reference's PAAC+FiGAR hot path — TEST INFRASTRUCTURE ONLY.

This package is the parity oracle (and, timed, the "port" CPU baseline). Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import it, and only as the checker
or the baseline — never as the thing measured or shipped. The product path
(manette_amd/ + libmanette_hip.so) never imports it.

Every function cites the reference file:line it restates (paths relative to the reference
repo andres-quintela/manette). Pinning (see DESIGN.md "Oracle"):
  * host loop, runner bookkeeping, tab_rep, sampling, returns: bit-exact against golden
    vectors produced by running the reference's own Python (tests/golden/make_golden.py);
  * preprocess: bit-exact against the reference's atari_emulator.py run on a fake ALE;
  * network/loss/optimizer constants: pinned by the TF graphs in pretrained/*/*.meta
    (tests/golden/meta_graph.json); the TF1 kernel arithmetic itself is unpinned (TF absent),
    so the math is restated from the graph structure and cross-checked against torch autograd.
"""
