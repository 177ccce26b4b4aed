set -e
cd $GRAFT_REPO_ROOT/tools/probes
for g in 768 1024 1280 2048; do timeout -k 10 60 ./mx_proto_m0 8 20 $g | grep -v mismatch; done
