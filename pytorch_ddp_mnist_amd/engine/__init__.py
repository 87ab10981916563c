"""Training engines: native MI355X step runtime and the torch-CPU reference engine."""
