# round 3 (session 2): PMC traffic of the C4 GMRES kernels and C5's 27-point passes (FETCH/WRITE + calibration)
cd /root/repo
(while true; do date > gpurun_out/hb; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
TAG=c4 REGEX='mdot|maxpy|zmc|stream_read' PMC_PASSES="FETCH_SIZE;WRITE_SIZE" bash tools/pmc_kernels.sh python3 $GRAFT_REPO_ROOT/tools/gmres_trace.py 256 60 || exit 1
TAG=c5 REGEX='zm27|cg_pb|stream_read' PMC_PASSES="FETCH_SIZE;WRITE_SIZE" bash tools/pmc_kernels.sh python3 $GRAFT_REPO_ROOT/tools/c5_trace.py 60 || exit 1
TAG=calib REGEX='stream_read' PMC_PASSES="FETCH_SIZE" bash tools/pmc_kernels.sh python3 $GRAFT_REPO_ROOT/tools/calib_stream.py || exit 1
echo all done
