"""Stub of r2r_src/env.py (imports MatterSim and loads depth .npy at import): the golden generator
drives the agent with dasa_amd.synth.SynthR2RBatch instead."""


class R2RBatch:
    pass
