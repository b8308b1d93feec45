set -u
bash tools/ab_run.sh r2d C2,C2main,C5,C3 ab/cur.so ab/stage16.so ab/stage32.so ab/nogen.so && \
bash tools/pmc_traffic.sh r2d_pmc "C2" ab/cur.so ab/stage16.so ab/stage32.so
