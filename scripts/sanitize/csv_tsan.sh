#!/bin/bash
# Host-only ThreadSanitizer run of the multi-threaded CSV tokenizer (csrc/csv_parser.cpp): 60k rows on 8 threads.
# MEASURED (r6, after the per-thread column tallies): no TSan reports; before, the threads added into the shared
# Col::n_text / n_num counters.
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
O=${TMPDIR:-/tmp}/csv_tsan
g++ -O1 -g -fsanitize=thread -std=c++17 -pthread -I $R/llama_github_io_amd/csrc $R/scripts/sanitize/csv_tsan_main.cpp \
    $R/llama_github_io_amd/csrc/csv_parser.cpp -o $O
$O
