# source this in a GPU script: a background writer keeps gpurun's silence watchdog informed
# while a long single test runs (the test's own timeout still bounds it)
( while true; do date +%s >> gpurun_out/.heartbeat; sleep 50; done ) &
HB_PID=$!
trap "kill $HB_PID 2>/dev/null" EXIT
