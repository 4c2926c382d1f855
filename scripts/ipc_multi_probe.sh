#!/bin/bash
# two processes on one GPU: exporter + importer, bounded by timeouts
set -u
nb=$1; mb=$2; d=$(mktemp -d /tmp/ipcprobe.XXXX)
timeout -k 5 90 ./scripts/ipc_multi_probe 0 $d $nb $mb & e=$!
timeout -k 5 80 ./scripts/ipc_multi_probe 1 $d $nb $mb; ri=$?
wait $e; re=$?
echo "nb=$nb mb=$mb importer=$ri exporter=$re"
rm -rf $d
[ $ri -eq 0 ]
