#!/bin/bash
# Host-only ASan+UBSan and TSan runs of the multi-threaded TreeSHAP (csrc/treeshap.cpp) on random forests with NA
# directions and categorical splits; the harness checks SHAP additivity for every row. MEASURED (r6): clean, max
# |sum(phi) + bias - prediction| 1e-15.
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
O=${TMPDIR:-/tmp}
g++ -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -std=c++17 -pthread $R/scripts/sanitize/treeshap_main.cpp \
    $R/llama_github_io_amd/csrc/treeshap.cpp -o $O/shap_asan
$O/shap_asan
g++ -O1 -g -fsanitize=thread -std=c++17 -pthread $R/scripts/sanitize/treeshap_main.cpp $R/llama_github_io_amd/csrc/treeshap.cpp -o $O/shap_tsan
$O/shap_tsan
