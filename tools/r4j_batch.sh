#!/bin/bash
# round-4 final-tree validation: every GPU test, smoke, the default bench line, its rocprof
# stats, and the STFT traffic passes of the shipped build.
set -o pipefail
bash tools/gpu_measure.sh r4j tests smoke bench prof pmcaux
