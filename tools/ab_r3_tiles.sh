set -e
for k in tb3r1w8 tb3 tb3r1w16; do EXTRA="--kernel $k" timeout -k 10 200 tools/ab_tb3_abl.sh 2 new1 new2; done
for k in tb3 tb3r1w8; do EXTRA="--kernel $k --dtype fp32 --scheme delta" timeout -k 10 200 tools/ab_tb3_abl.sh 2 old new1 new2; done
