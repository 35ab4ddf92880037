set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 5 60 rocprofv3 -L > gpurun_out/pmc/list.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*\|TCC_[A-Z_0-9]*\|TCP_[A-Z_0-9]*" gpurun_out/pmc/list.txt | sort -u > gpurun_out/pmc/names.txt
wc -l gpurun_out/pmc/names.txt
