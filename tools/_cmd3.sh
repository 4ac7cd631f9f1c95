bash tools/_cmd.sh || exit $?
bash tools/_cmd2.sh
