"""Reference-API mirror of DASA's r2r_src policy modules (agent_dg, model, vilmodel, r2rmodel, param)
running on the MI355X HIP kernels of libdasa_hip.so. Class names, constructor/forward signatures and
state_dict keys match the reference so train.py and reference checkpoints work unchanged."""
