#!/bin/bash
set -o pipefail
bash tools/r04_gpu5.sh && bash tools/r04_gpu4.sh
