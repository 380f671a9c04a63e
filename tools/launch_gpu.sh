#!/bin/bash
# Start one gpurun call in the background (this container side): its output
# goes to gpurun_out/<name>.txt. Usage: tools/launch_gpu.sh NAME 'command'
name=$1; shift
nohup /usr/local/graft/bin/gpurun --timeout 1200 -- "$@" > "gpurun_out/$name.txt" 2>&1 &
echo "started $name (pid $!)"
