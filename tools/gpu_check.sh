cd $GRAFT_REPO_ROOT
bash tools/scan.sh 2 "4096 65536 262144 1048576" oneshot
bash tools/scan.sh 2 "4096 65536 262144 1048576" mesh
bash tools/scan.sh 2 "4096 65536 262144 1048576" ring
