#!/bin/bash
# Runs tools/vmem_import_probe (two processes on GPU 0); output: gpurun_out/vmem/{exporter,importer}.jsonl
set -o pipefail
mkdir -p gpurun_out/vmem
name="p$$"
timeout -k 10 90 tools/vmem_import_probe exporter "$name" > gpurun_out/vmem/exporter.jsonl 2>&1 &
ep=$!
sleep 1
timeout -k 10 90 tools/vmem_import_probe importer "$name" > gpurun_out/vmem/importer.jsonl 2>&1
irc=$?
wait $ep
erc=$?
rm -f /dev/shm/rdc_vmem_$name
cat gpurun_out/vmem/exporter.jsonl gpurun_out/vmem/importer.jsonl
echo "{\"importer_rc\": $irc, \"exporter_rc\": $erc}"
[ $irc -eq 0 ] && [ $erc -eq 0 ]
