# shared by the fleet scripts: HOSTS=(...) from the ansible inventory
INV=${INV:-./deploy/ansible_hosts.ini}
GROUP=${GROUP:-thinvids_workers}
mapfile -t HOSTS < <(ansible -i "$INV" --list-hosts "$GROUP" | awk 'NR>1{print $1}')
if ((${#HOSTS[@]} == 0)); then echo "no hosts in group '$GROUP' of '$INV'" >&2; exit 1; fi
valid_host() { [[ $1 =~ ^[A-Za-z0-9._-]+$ ]]; }
