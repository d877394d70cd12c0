"""oracle/ — TEST INFRASTRUCTURE (the parity checker). Never the product path.

CPU restatement of the reference U-RED hot path:
  nn_oracle.c / nn_ref.py : the DCD chamfer3D nearest-neighbour kernels
  ured_ref.py             : TargetEncoder / re_residual_net / DeformNet_MatchingNet
                            forward, get_part / get_shape / losses, the train step.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import it.
Pinned against golden vectors generated from the reference itself
(tests/golden/make_golden.py, run in the survey container where the reference's
pure-torch modules import).
"""
