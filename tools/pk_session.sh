set -o pipefail
LIBS="cur ff4 ff8 ff100000" VARS=0:0:0,66:8:8 bash tools/pk_ab.sh || exit 1
LIBS="cur ff4 ff100000" VARS=0:0:0,66:8:8 SCS=readme RND=1 bash tools/pk_ab.sh || exit 1
LIBS="cur ff4 ff100000" VARS=0:0:0,66:8:8 SCS="readme cfg5" bash tools/pk_ab.sh
