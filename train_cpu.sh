#!/bin/bash
# Single-process plumbing run (reference train_cpu.sh).
python ddp_tutorial_cpu.py "$@"
