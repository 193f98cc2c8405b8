#!/bin/bash
# Host-only AddressSanitizer + UBSan run of the CSV tokenizer over edge-case inputs (empty, unterminated quotes,
# ragged rows, CRLF, escaped quotes, a 30k-row quoted file), each in an exact-size heap buffer.
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
O=${TMPDIR:-/tmp}/csv_asan
g++ -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -std=c++17 -pthread -I $R/llama_github_io_amd/csrc \
    $R/scripts/sanitize/csv_asan_main.cpp $R/llama_github_io_amd/csrc/csv_parser.cpp -o $O
$O
